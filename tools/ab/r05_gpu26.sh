#!/bin/bash
# chunk-span statistics of every MSM's runs in one C4 step (TNS_FIX_STATS=1), to explain the second opening's fixup
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu26
mkdir -p $out
TNS_FIX_STATS=1 timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 1 --warmup 0 --no-extras --stage-steps 0 > $out/bench.jsonl 2> $out/stats.txt || { tail -20 $out/stats.txt; exit 1; }
grep fix-stats $out/stats.txt | head -20
