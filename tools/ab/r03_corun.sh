#!/bin/bash
# round-3: the co-running sort (second MSM of a pair sorting under the first's accumulation):
# parity under TNS_MSM_STAGGER=1, then the C4 bench A/B (default / stagger + co-running kernels /
# a resident-only accumulation grid; the co-running kernels were measured and removed)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${OUT:-r03corun}
mkdir -p $out
if [ -n "${TESTS:-}" ]; then
TNS_MSM_STAGGER=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$TESTS" > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc = 0 ] || { grep -E "Error|assert|FAILED" $out/pytest.log | head -20; exit $rc; }
fi
AB="${AB:--;TNS_MSM_STAGGER=1;TNS_MSM_STAGGER=1 TNS_ACC_WAVES=3}" OUT=${OUT:-r03corun} STEPS=${STEPS:-10} TESTS= bash tools/ab/r03_ab.sh
