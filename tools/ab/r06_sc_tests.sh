#!/bin/bash
# round 6: the generic sum-check GPU tests (fold-oracle parity, every schedule regime, host rounds)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06_sc_tests
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sumcheck.py > gpurun_out/r06_sc_tests/pytest.txt 2>&1 || { tail -30 gpurun_out/r06_sc_tests/pytest.txt; exit 1; }
tail -2 gpurun_out/r06_sc_tests/pytest.txt
