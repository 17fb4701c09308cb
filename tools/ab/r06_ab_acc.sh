#!/bin/bash
# round 6: when the first opening accumulation starts (TNS_ACC_AFTER build variants: 0 = after both
# sorts, 1 = after its own sort, 2 = after the other lane's second pass), C4 A/B + timelines
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/ab/r06_ab_lib.sh accafter 3 aa1 aa2 || exit 1
L=$GRAFT_REPO_ROOT/multilinear-map-cryptography_amd
for v in aa1 aa2; do
  out=gpurun_out/r06_ab_accafter/tr_$v
  TNS_LIB=$L/libtns_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out -o run --output-format csv -- python3 bench.py --no-extras --steps 2 --warmup 1 > $out.log 2>&1 || exit 1
  f=$(find $out -name "run_kernel_trace.csv" | head -n 1)
  python3 tools/trace_tail.py "$f" k_u64_tables 0.05 > gpurun_out/r06_ab_accafter/timeline_$v.txt 2>&1
done
