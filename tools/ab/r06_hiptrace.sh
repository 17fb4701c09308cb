#!/bin/bash
# round 6: kernel + HIP API trace of two C4 steps (the host turns between device phases)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06_hiptrace
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d $out/tr -o run --output-format csv -- python3 bench.py --no-extras --steps 2 --warmup 1 > $out/run.log 2>&1 || { tail -20 $out/run.log; exit 1; }
ls -R $out/tr | head -20
