#!/bin/bash
# round 5 GPU pass 21: rotating point sums (default) vs x-indexed updates (libtns_r0) -- sum-check tests,
# timings, SQ instruction counts
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu21
mkdir -p $out
L=$GRAFT_REPO_ROOT/multilinear-map-cryptography_amd
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sumcheck.py tests/test_gpu_parity.py -k "sumcheck" > $out/pytest_sc.txt 2>&1 || { tail -30 $out/pytest_sc.txt; exit 1; }
tail -1 $out/pytest_sc.txt
for rep in 1 2 3; do
  for v in default r0; do
    if [ $v = default ]; then lib=$L/libtns.so; else lib=$L/libtns_$v.so; fi
    TNS_LIB=$lib timeout -k 10 200 python3 -u tools/sc_bench.py 20,24 > $out/sc_${v}_$rep.json 2> $out/sc_${v}_$rep.err || { cat $out/sc_${v}_$rep.err; exit 1; }
    echo "$v $rep $(python3 -c "import json; d=json.load(open('$out/sc_${v}_$rep.json')); print({k: (v['ms'], v['kernel_ms']) for k, v in d.items()})")"
  done
done
for v in default r0; do
  if [ $v = default ]; then lib=$L/libtns.so; else lib=$L/libtns_$v.so; fi
  TNS_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU -d $out/pmc_$v -o run --output-format csv -- python3 tools/sc_bench.py 24 > $out/pmc_$v.log 2>&1 || exit 1
  echo "== $v"; python3 tools/pmc_view.py $(ls $out/pmc_$v/*counter_collection.csv | head -1) k_sc_round_poly
done
