#!/bin/bash
# round 5 GPU pass 7: sum-check round kernel with 32-bit composition flags (scalar loads) --
# parity tests, then variants alternating (unrolled / point loop / 4 waves / L2 touch / LDS staging /
# hand-written composition), SQ counters and a kernel trace of the point-loop build
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu7
mkdir -p $out
L=$GRAFT_REPO_ROOT/multilinear-map-cryptography_amd
TNS_LIB=$L/libtns_uix.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sumcheck.py tests/test_gpu_parity.py -k "sumcheck" > $out/pytest_sc_uix.txt 2>&1 || { tail -30 $out/pytest_sc_uix.txt; exit 1; }
tail -1 $out/pytest_sc_uix.txt
for rep in 1 2 3; do
  for v in ui uix uix4 uixp uisx hand; do
    TNS_LIB=$L/libtns_$v.so timeout -k 10 200 python3 -u tools/sc_bench.py 20,24 > $out/sc_${v}_$rep.json 2> $out/sc_${v}_$rep.err || { cat $out/sc_${v}_$rep.err; exit 1; }
    echo "$v $rep $(python3 -c "import json; d=json.load(open('$out/sc_${v}_$rep.json')); print({k: (v['ms'], v['kernel_ms'], v['hbm_frac']) for k, v in d.items()})")"
  done
done
TNS_LIB=$L/libtns_uix.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM -d $out/pmc_uix -o run --output-format csv -- python3 tools/sc_bench.py 24 > $out/pmc_uix.log 2>&1 || exit 1
python3 tools/pmc_view.py $(ls $out/pmc_uix/*counter_collection.csv | head -1) k_sc_round_poly
TNS_LIB=$L/libtns_uix.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/trace_uix -o run --output-format csv -- python3 tools/sc_bench.py 20,24 > $out/trace_uix.log 2>&1 || exit 1
for s in 18 20; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/c2_srs$s -o run --output-format csv -- python3 tools/msm_trace.py 20 20 $s > $out/c2_srs$s.log 2>&1 || exit 1
  tail -n 1 $out/c2_srs$s.log
done
