#!/bin/bash
# round 4: second-level bucket reduction (k_reduce_level2) A/B -- C2 MSM (2^20, table plan) and the
# C4 bench, default vs TNS_RED_L1=0 (masked sums straight over the first level's groups)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04_red2
mkdir -p $out
for rep in 1 2; do
  for v in "TNS_RED_L1=0" "TNS_RED_L1=4" "TNS_RED_L1=8"; do
    env $v timeout -k 10 120 python3 tools/msm_trace.py 20 20 > $out/c2_${v}_$rep.txt 2>&1 || exit $?
    echo "$v rep $rep: $(tail -n 1 $out/c2_${v}_$rep.txt)"
  done
done
for v in "TNS_RED_L1=0" "TNS_RED_L1=4"; do
  env $v timeout -k 10 200 python3 -u bench.py --no-extras --steps 10 --warmup 3 > $out/c4_$v.jsonl 2> $out/c4_$v.err || exit $?
  echo "$v C4: $(python3 -c "import json,sys; d=json.loads(open('$out/c4_$v.jsonl').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['stages_ms_per_step'])")"
done
