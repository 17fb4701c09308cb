#!/bin/bash
# GPU tests, then the quotient-pass histogram A/B, then the SQ issue counters of one C4 step
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/qh
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/qh/pytest.log 2>&1; tail -2 gpurun_out/qh/pytest.log
bash tools/ab/ab_env.sh X=1 TNS_NO_QUOTIENT_HIST=1 X=2 TNS_NO_QUOTIENT_HIST=1
bash tools/pmc_sq.sh r02
