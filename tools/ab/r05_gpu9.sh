#!/bin/bash
# round 5 GPU pass 9: fold-round load order (AHEAD 0 / 1 = default / 2), parity tests on the default
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu9
mkdir -p $out
L=$GRAFT_REPO_ROOT/multilinear-map-cryptography_amd
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sumcheck.py tests/test_gpu_parity.py -k "sumcheck" > $out/pytest_sc.txt 2>&1 || { tail -30 $out/pytest_sc.txt; exit 1; }
tail -1 $out/pytest_sc.txt
for rep in 1 2 3; do
  for v in default a0 a2 hand; do
    if [ $v = default ]; then lib=$L/libtns.so; else lib=$L/libtns_$v.so; fi
    TNS_LIB=$lib timeout -k 10 200 python3 -u tools/sc_bench.py 20,24 > $out/sc_${v}_$rep.json 2> $out/sc_${v}_$rep.err || { cat $out/sc_${v}_$rep.err; exit 1; }
    echo "$v $rep $(python3 -c "import json; d=json.load(open('$out/sc_${v}_$rep.json')); print({k: (v['ms'], v['kernel_ms'], v['hbm_frac']) for k, v in d.items()})")"
  done
done
for v in a2; do
TNS_LIB=$L/libtns_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/trace_$v -o run --output-format csv -- python3 tools/sc_bench.py 20,24 > $out/trace_$v.log 2>&1 || exit 1
done
for s in 18 20; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/c2_srs$s -o run --output-format csv -- python3 tools/msm_trace.py 20 20 $s > $out/c2_srs$s.log 2>&1 || exit 1
  grep "msm 2" $out/c2_srs$s.log
done
