#!/bin/bash
# kernel trace of the C4 bench (2 timed steps) and the step timeline from the last proof's
# address-table kernel on: tools/c4_step_trace.sh <tag> [VAR=val ...]
set -uo pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/c4trace_$tag
mkdir -p $out
for e in "$@"; do export "$e"; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/tr -o run --output-format csv -- python3 bench.py --no-extras --steps 2 --warmup 1 > $out/run.log 2>&1 || exit $?
f=$(find $out/tr -name "run_kernel_trace.csv" | head -n 1)
python3 tools/trace_tail.py "$f" k_u64_tables 0.05 > $out/tail.txt 2>&1
tail -n 25 $out/tail.txt
