#!/bin/bash
# Kernel-trace statistics and HBM traffic counters for the C4 bench (run on the GPU box).
#   tools/profile_round.sh <tag> [bench args...]
# Pass 1: rocprofv3 --kernel-trace --stats.  Passes 2/3: --pmc FETCH_SIZE, --pmc WRITE_SIZE
# (separate passes: the two do not fit one TCC pass on gfx950; no trace domains beside PMC).
set -euo pipefail
tag=${1:-r01}; shift || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/prof_$tag
mkdir -p $out
args=("--no-extras" "--steps" "2" "--warmup" "1" "$@")
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/ks -o run --output-format csv -- python3 bench.py "${args[@]}" > $out/ks.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o run --output-format csv -- python3 bench.py "${args[@]}" > $out/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $out/write -o run --output-format csv -- python3 bench.py "${args[@]}" > $out/write.log 2>&1
find $out -name "*.csv" | head -20
