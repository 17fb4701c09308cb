#!/bin/bash
# round 5 GPU pass 10: four-lanes-a-pair small-round kernel (parity, range A/B); C2 table window 20
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu10
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sumcheck.py tests/test_gpu_parity.py -k "sumcheck" > $out/pytest_sc.txt 2>&1 || { tail -30 $out/pytest_sc.txt; exit 1; }
tail -1 $out/pytest_sc.txt
TNS_SC_SPLIT_LOG=20 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sumcheck.py tests/test_gpu_parity.py -k "sumcheck" > $out/pytest_sc_all_split.txt 2>&1 || { tail -30 $out/pytest_sc_all_split.txt; exit 1; }
tail -1 $out/pytest_sc_all_split.txt
for rep in 1 2; do
  for v in 0 12 14 16 18; do
    TNS_SC_SPLIT_LOG=$v timeout -k 10 200 python3 -u tools/sc_bench.py 20,24 > $out/sc_${v}_$rep.json 2> $out/sc_${v}_$rep.err || { cat $out/sc_${v}_$rep.err; exit 1; }
    echo "split<=2^$v $rep $(python3 -c "import json; d=json.load(open('$out/sc_${v}_$rep.json')); print({k: (v['ms'], v['kernel_ms'], v['hbm_frac']) for k, v in d.items()})")"
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 tools/sc_bench.py 20,24 > $out/trace.log 2>&1 || exit 1
for c in 19 20; do
  TNS_TABLE_C=$c timeout -k 10 120 python3 tools/msm_trace.py 20 20 18 > $out/c2_c$c.log 2>&1 || exit 1
  echo "TNS_TABLE_C=$c $(grep 'msm 2' $out/c2_c$c.log)"
done
