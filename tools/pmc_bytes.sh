#!/bin/bash
# FETCH_SIZE and WRITE_SIZE per kernel for one C4 step (two separate --pmc passes): tools/pmc_bytes.sh <tag>
set -euo pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in FETCH_SIZE WRITE_SIZE; do
  out=gpurun_out/pmcb_${tag}_$c
  mkdir -p $out
  timeout -s KILL 300 rocprofv3 --pmc $c -d $out -o run --output-format csv -- python3 bench.py --no-extras --steps 1 --warmup 0 > $out/bench.log 2>&1
done
