#!/bin/bash
# round 6: the generic sum-check at 2^20 -- Python vs bare C call wall, and a kernel trace of it
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06_sc_$1
mkdir -p $out
timeout -k 10 120 python3 tools/sc_trace.py 20 30 > $out/wall.txt 2>&1 || { cat $out/wall.txt; exit 1; }
cat $out/wall.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/tr -o run --output-format csv -- python3 tools/sc_trace.py 20 3 > $out/trace_run.log 2>&1 || exit 1
f=$(find $out/tr -name "run_kernel_trace.csv" | head -n 1)
python3 tools/trace_tail.py "$f" "round_poly<false" 0 > $out/timeline_all.txt 2>&1
tail -n 40 $out/timeline_all.txt
