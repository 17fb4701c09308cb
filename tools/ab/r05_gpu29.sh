#!/bin/bash
# MSM sort variants incl. the per-call geometry / readback knobs, then the bench at the driver's arguments
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu29
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "sort_variants" > $out/pytest.txt 2>&1 || { tail -30 $out/pytest.txt; exit 1; }
tail -1 $out/pytest.txt
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.jsonl 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
tail -n 1 $out/bench.jsonl | cut -c1-200
