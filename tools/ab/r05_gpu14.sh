#!/bin/bash
# round 5 GPU pass 14: persistent sum-check tail (parity tests incl. the error paths; TNS_SC_TAIL_LOG A/B)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu14
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sumcheck.py tests/test_gpu_parity.py -k "sumcheck" > $out/pytest_sc.txt 2>&1 || { tail -30 $out/pytest_sc.txt; exit 1; }
tail -1 $out/pytest_sc.txt
TNS_SC_TAIL_LOG=18 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sumcheck.py tests/test_gpu_parity.py -k "sumcheck" > $out/pytest_sc_tail18.txt 2>&1 || { tail -30 $out/pytest_sc_tail18.txt; exit 1; }
tail -1 $out/pytest_sc_tail18.txt
for rep in 1 2; do
  for v in 13 0 11 15 17; do
    TNS_SC_TAIL_LOG=$v timeout -k 10 200 python3 -u tools/sc_bench.py 20,24 > $out/sc_${v}_$rep.json 2> $out/sc_${v}_$rep.err || { cat $out/sc_${v}_$rep.err; exit 1; }
    echo "tail<=2^$v $rep $(python3 -c "import json; d=json.load(open('$out/sc_${v}_$rep.json')); print({k: (v['ms'], v['kernel_ms'], v['hbm_frac']) for k, v in d.items()})")"
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 tools/sc_bench.py 20,24 > $out/trace.log 2>&1 || exit 1
