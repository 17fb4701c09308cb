#!/bin/bash
# round 6: the sum-check's last rounds on the host (SC_HOST_PAIRS 0 / 16 / 32 / 64): parity of the
# default build's sum-check and proof tests, then the A/B
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06_ab_hp
TNS_LIB=$GRAFT_REPO_ROOT/multilinear-map-cryptography_amd/libtns_hp32.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sumcheck.py tests/test_gpu_parity.py > gpurun_out/r06_ab_hp/tests.txt 2>&1 || { tail -30 gpurun_out/r06_ab_hp/tests.txt; exit 1; }
tail -3 gpurun_out/r06_ab_hp/tests.txt
bash tools/ab/r06_ab_sc.sh 2 hp0 hp16 hp32 hp64
