#!/bin/bash
# round 5 GPU pass 5: LDS-staged sum-check round kernel (tests; staged / unstaged x 4 / 3 waves),
# C2 allocation-order test
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu5
mkdir -p $out
L=$GRAFT_REPO_ROOT/multilinear-map-cryptography_amd
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sumcheck.py tests/test_gpu_parity.py -k "sumcheck" > $out/pytest_sc.txt 2>&1 || { tail -30 $out/pytest_sc.txt; exit 1; }
tail -2 $out/pytest_sc.txt
for rep in 1 2; do
  for v in default sc3 nostage nostage3; do
    if [ $v = default ]; then lib=$L/libtns.so; else lib=$L/libtns_$v.so; fi
    TNS_LIB=$lib timeout -k 10 200 python3 -u tools/sc_bench.py 20,24 > $out/sc_${v}_$rep.json 2> $out/sc_${v}_$rep.err || { cat $out/sc_${v}_$rep.err; exit 1; }
    echo "$v $rep $(python3 -c "import json; d=json.load(open('$out/sc_${v}_$rep.json')); print({k: (v['ms'], v['kernel_ms'], v['hbm_frac']) for k, v in d.items()})")"
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/sc_trace -o run --output-format csv -- python3 tools/sc_bench.py 20,24 > $out/sc_trace.log 2>&1 || exit 1
for m in none lagrange_first table_first; do
  timeout -k 10 200 python3 -u tools/c2_alloc.py $m > $out/c2_$m.json 2> $out/c2_$m.err || { tail $out/c2_$m.err; exit 1; }
  cat $out/c2_$m.json
  TNS_TABLE_CONTIG=1 timeout -k 10 200 python3 -u tools/c2_alloc.py $m > $out/c2c_$m.json 2> $out/c2c_$m.err || { tail $out/c2c_$m.err; exit 1; }
  cat $out/c2c_$m.json
done
