#!/bin/bash
# round 6: k_accumulate flags whether any 8-chunk group lies inside one bucket; without one every
# k_fix_level launch returns at once (gf build): parity (skewed and uniform MSMs), C4 / drop-in /
# C2 A/B (tools/ab/r06_ab_dropin.sh), C2 timeline
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/multilinear-map-cryptography_amd
out=gpurun_out/r06_ab_groupflag
mkdir -p $out
TNS_LIB=$L/libtns_gf.so timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_lagrange.py tests/test_gpu_sharded.py tests/test_gpu_routes.py > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
AB_SUFFIX=_gf bash tools/ab/r06_ab_dropin.sh 3 gf || exit 1
