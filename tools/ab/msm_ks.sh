#!/bin/bash
# kernel trace of standalone MSMs: tools/ab/msm_ks.sh <tag> <log_n> [VAR=val ...]
set -euo pipefail
tag=$1; k=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for e in "$@"; do export "$e"; done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/msm_$tag -o run --output-format csv -- python3 tools/msm_trace.py $k 3 > gpurun_out/msm_$tag.log 2>&1
tail -c 300 gpurun_out/msm_$tag.log
