#!/bin/bash
# round 6: the bench as the driver runs it (N = 1, all extras), then the 4-rank sharded rehearsal on one
# GPU (gloo exchange): tools/ab/r06_bench_full.sh <tag> [no-rehearsal]
set -uo pipefail
tag=$1; norh=${2:-}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06_full_$tag
mkdir -p $out
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $out/bench.jsonl 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 - "$out/bench.jsonl" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
keys = ["ms_per_step", "value", "ms_per_step_dropin", "ms_per_step_no_table", "no_table_same_proof", "c5_one_gpu_ms_per_step",
        "msm_ms_2^20", "msm_ms_2^20_no_table", "shout_ms_2^20", "twist_last_prove_ms"]
print({k: d.get(k) for k in keys})
print("sumcheck", {k: v.get("ms") for k, v in (d.get("sumcheck_generic") or {}).items() if isinstance(v, dict)})
print("cpu", (d.get("cpu_baseline") or {}).get("value"), "roof", d["roofline"].get("frac"), d["roofline"].get("avg_launch_ms"))
PY
[ -n "$norh" ] && exit 0
timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --gpus 4 --steps 3 --warmup 1 --rehearse-one-gpu > $out/rehearse4.jsonl 2> $out/rehearse4.err || { tail -20 $out/rehearse4.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$out/rehearse4.jsonl').read().strip().splitlines()[-1])
print('rehearse4', d['ms_per_step'], d['value'], [(r['exchanges_per_step'], r['mean_exchange_us'], r['mean_exchange_bytes_per_rank']) for r in d['comm']['per_rank']])"
