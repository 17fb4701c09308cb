#!/bin/bash
# early-clobber fix: the chain probe, madd throughput old vs new asm operands, then the bench
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03ec
mkdir -p $out
timeout -k 10 120 tools/chainfuse > $out/chainfuse.txt 2>&1 || { echo "probe rc=$?"; exit 1; }
grep "finish2(icp)\|node0 limbs" $out/chainfuse.txt
for i in 1 2; do
  timeout -k 10 60 tools/maddbench_old ec_old >> $out/maddbench.txt 2>&1 || exit 1
  timeout -k 10 60 tools/maddbench ec_new >> $out/maddbench.txt 2>&1 || exit 1
done
cat $out/maddbench.txt
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --no-extras > $out/bench.jsonl 2> $out/bench.err
echo "bench rc=$?"
python3 -c "import json;d=json.loads(open('$out/bench.jsonl').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['stages_ms_per_step'])"
