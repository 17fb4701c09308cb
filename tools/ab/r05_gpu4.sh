#!/bin/bash
# round 5 GPU pass 4: lazy-domain sum-check kernel (tests; 4 vs 3 waves), C2/C3 table-window A/B
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu4
mkdir -p $out
L=$GRAFT_REPO_ROOT/multilinear-map-cryptography_amd
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sumcheck.py tests/test_gpu_parity.py -k "sumcheck" > $out/pytest_sc.txt 2>&1 || { tail -30 $out/pytest_sc.txt; exit 1; }
tail -2 $out/pytest_sc.txt
for rep in 1 2; do
  for v in default sc3; do
    if [ $v = default ]; then lib=$L/libtns.so; else lib=$L/libtns_$v.so; fi
    TNS_LIB=$lib timeout -k 10 200 python3 -u tools/sc_bench.py 20,24 > $out/sc_${v}_$rep.json 2> $out/sc_${v}_$rep.err || { cat $out/sc_${v}_$rep.err; exit 1; }
    echo "$v $rep $(cat $out/sc_${v}_$rep.json | cut -c1-400)"
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/sc_trace -o run --output-format csv -- python3 tools/sc_bench.py 20,24 > $out/sc_trace.log 2>&1 || exit 1
for rep in 1 2; do
  for e in TNS_AB_DEFAULT=1 TNS_TABLE_C=22 TNS_TABLE_C=21; do
    env $e timeout -k 10 200 python3 -u tools/c2c3_bench.py > $out/c2c3_${e}_$rep.json 2> $out/c2c3_${e}_$rep.err || { tail $out/c2c3_${e}_$rep.err; exit 1; }
    echo "$e $rep $(cat $out/c2c3_${e}_$rep.json)"
  done
done
