#!/bin/bash
# round 4: kernel traces of the C4 bench, default schedule vs TNS_MSM_STAGGER=1 (lane 1's opening
# sort with the 2048-tile co-running kernels under lane 0's accumulation), for the step timeline
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04_stagger
mkdir -p $out
args=("--no-extras" "--steps" "2" "--warmup" "1")
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/def -o run --output-format csv -- python3 bench.py "${args[@]}" > $out/def.log 2>&1 || exit $?
TNS_MSM_STAGGER=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/stg -o run --output-format csv -- python3 bench.py "${args[@]}" > $out/stg.log 2>&1 || exit $?
for v in def stg; do
  f=$(find $out/$v -name "run_kernel_trace.csv" | head -n 1)
  python3 tools/trace_tail.py "$f" k_u64_tables 0.05 > $out/${v}_tail.txt 2>&1 || true
done
echo done
