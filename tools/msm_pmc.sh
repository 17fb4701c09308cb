#!/bin/bash
# SQ counters of the standalone 2^k MSM's kernels: tools/msm_pmc.sh <tag> <log_n> "<counters>"
set -euo pipefail
tag=$1; k=$2; ctrs=$3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc $ctrs -d gpurun_out/pmc_$tag -o run --output-format csv -- python3 tools/msm_trace.py $k 1 > gpurun_out/pmc_$tag.log 2>&1
find gpurun_out/pmc_$tag -name "*counter_collection.csv" | head -1
