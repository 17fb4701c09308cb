#!/bin/bash
# One GPU call: parity tests, the default bench line, and a rocprofv3 kernel-trace summary.
#   tools/ab/gpu_round.sh <tag>
set -euo pipefail
tag=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/round_$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1
tail -3 $out/pytest_gpu.log
timeout -k 10 300 python -u bench.py > $out/bench.jsonl 2> $out/bench.err
cat $out/bench.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/ks -o run --output-format csv -- python3 bench.py --no-extras --steps 2 --warmup 1 > $out/ks.log 2>&1
find $out/ks -name "*stats*"
