#!/bin/bash
# kernel trace of a short C4 bench under an environment setting: tools/ab/ks_env.sh <tag> [VAR=val ...]
set -euo pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for e in "$@"; do export "$e"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ks_$tag -o run --output-format csv -- python3 bench.py --no-extras --steps 2 --warmup 1 > gpurun_out/ks_$tag.log 2>&1
tail -c 400 gpurun_out/ks_$tag.log
