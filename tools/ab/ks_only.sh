#!/bin/bash
# rocprofv3 kernel trace + stats of a short C4 bench: tools/ab/ks_only.sh <tag> [bench args...]
set -euo pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/ks_$tag
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out -o run --output-format csv -- python3 bench.py --no-extras --steps 2 --warmup 1 "$@" > $out/bench.log 2>&1
tail -c 1500 $out/bench.log
