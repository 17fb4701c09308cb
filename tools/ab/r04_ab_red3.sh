#!/bin/bash
# round 4: bucket-reduction tuning with the second level -- C2 kernel trace, C4 with TNS_RED_L 4/8/16
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04_red3
mkdir -p $out
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/c2ks -o run --output-format csv -- python3 tools/msm_trace.py 20 3 > $out/c2ks.log 2>&1 || exit $?
f=$(find $out/c2ks -name "run_kernel_trace.csv" | head -n 1)
python3 tools/trace_tail.py "$f" k_scalar_bits > $out/c2_tail.txt 2>&1
for rep in 1 2; do
  for v in "TNS_RED_L=16" "TNS_RED_L=8" "TNS_RED_L=4"; do
    env $v timeout -k 10 200 python3 -u bench.py --no-extras --steps 10 --warmup 3 > $out/c4_${v}_$rep.jsonl 2> $out/c4_${v}_$rep.err || exit $?
    echo "$v rep $rep C4: $(python3 -c "import json,sys; d=json.loads(open('$out/c4_${v}_$rep.jsonl').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['stages_ms_per_step']['msm_reduce'], d['stages_ms_per_step']['msm_fixup'])")"
  done
done
