#!/bin/bash
# sum-check schedule variants (per-call env knobs) against the oracle, then the whole GPU suite and smoke
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu28
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sumcheck.py > $out/pytest_sc.txt 2>&1 || { tail -30 $out/pytest_sc.txt; exit 1; }
tail -1 $out/pytest_sc.txt
timeout -k 10 1500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $out/pytest_gpu.txt 2>&1 || { tail -30 $out/pytest_gpu.txt; exit 1; }
tail -2 $out/pytest_gpu.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || { tail -20 $out/smoke.txt; exit 1; }
tail -1 $out/smoke.txt
