#!/bin/bash
# persistent-scatter A/B: GPU bucket-sort tests under TNS_BS_PERSIST=2, then C4 bench lines
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/persist
TNS_BS_PERSIST=2 timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "msm or twist" > gpurun_out/persist/pytest.log 2>&1; tail -2 gpurun_out/persist/pytest.log
bash tools/ab/ab_env.sh X=1 TNS_BS_PERSIST=1 TNS_BS_PERSIST=2 TNS_BS_PERSIST=3 X=2 TNS_BS_PERSIST=2
