#!/bin/bash
# LDS counters per kernel for one C4 step (bucket-sort diagnosis): tools/pmc_lds.sh <tag>
set -euo pipefail
tag=$1; shift || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/lds_$tag
mkdir -p $out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD -d $out -o run --output-format csv -- python3 bench.py --no-extras --steps 1 --warmup 0 --stage-steps 0 > $out/bench.log 2>&1
f=$(find $out -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import collections, csv, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if "k_bs_" not in k and "k_accumulate" not in k:
        continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in agg.items():
    w = max(1.0, c["SQ_WAVES"]); wc = max(1.0, c["SQ_WAVE_CYCLES"])
    print(f"{k[:44]:44s} lds_inst/wave {c['SQ_INSTS_LDS']/w:8.0f} bank_conflict/lds_inst {c['SQ_LDS_BANK_CONFLICT']/max(1,c['SQ_INSTS_LDS']):7.2f} "
          f"active_lds {c['SQ_ACTIVE_INST_LDS']/wc:5.2f} wait_lds {c['SQ_WAIT_INST_LDS']/wc:5.2f} vmem_wr/wave {c['SQ_INSTS_VMEM_WR']/w:7.0f} vmem_rd/wave {c['SQ_INSTS_VMEM_RD']/w:7.0f}")
PY
