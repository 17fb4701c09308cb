#!/bin/bash
# round 6: the sort segsetry's one-block kernels only up to 2^13 / 2^15 segments (TNS_SCAN_SMALL_LOG build variants; multi-block scans above): parity, C4 A/B, timelines
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/multilinear-map-cryptography_amd
out=gpurun_out/r06_ab_segs
mkdir -p $out
TNS_LIB=$L/libtns_$1.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_lagrange.py > $out/tests_$1.txt 2>&1 || { tail -30 $out/tests_$1.txt; exit 1; }
tail -1 $out/tests_$1.txt
bash tools/ab/r06_ab_lib.sh segs 5 "$@" || exit 1
for v in "$@"; do
  TNS_LIB=$L/libtns_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/tr_$v -o run --output-format csv -- python3 bench.py --no-extras --steps 2 --warmup 1 > $out/tr_$v.log 2>&1 || exit 1
  f=$(find $out/tr_$v -name "run_kernel_trace.csv" | head -n 1)
  python3 tools/trace_tail.py "$f" k_u64_tables 0.05 > $out/timeline_$v.txt 2>&1
done
