#!/bin/bash
# round 5 GPU pass 8: SQ counters and a kernel trace of the point-loop sum-check build; C2 traces
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu8
mkdir -p $out
L=$GRAFT_REPO_ROOT/multilinear-map-cryptography_amd
for v in uix hand; do
TNS_LIB=$L/libtns_$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM -d $out/pmc_$v -o run --output-format csv -- python3 tools/sc_bench.py 24 > $out/pmc_$v.log 2>&1 || exit 1
python3 tools/pmc_view.py $(ls $out/pmc_$v/*counter_collection.csv | head -1) k_sc_round_poly
TNS_LIB=$L/libtns_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/trace_$v -o run --output-format csv -- python3 tools/sc_bench.py 20,24 > $out/trace_$v.log 2>&1 || exit 1
done
for s in 18 20; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/c2_srs$s -o run --output-format csv -- python3 tools/msm_trace.py 20 20 $s > $out/c2_srs$s.log 2>&1 || exit 1
  tail -n 1 $out/c2_srs$s.log
done
