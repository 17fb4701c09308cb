#!/bin/bash
# SQ occupancy/issue counters per kernel for one C4 step: tools/pmc_sq.sh <tag> [bench args...]
set -euo pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/sq_$tag
mkdir -p $out
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $out -o run --output-format csv -- python3 bench.py --no-extras --steps 1 --warmup 0 "$@" > $out/bench.log 2>&1
