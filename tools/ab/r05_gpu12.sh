#!/bin/bash
# round 5 GPU pass 12: sum-check host turn without per-round inversions (PREQUEUE A/B, trace);
# table window without the near-tie rule (C2 / C3 and a 2^16 MSM vs the old windows); full GPU suite
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu12
mkdir -p $out
for rep in 1 2; do
  for v in 1 0; do
    TNS_SC_PREQUEUE=$v timeout -k 10 200 python3 -u tools/sc_bench.py 20,24 > $out/sc_${v}_$rep.json 2> $out/sc_${v}_$rep.err || { cat $out/sc_${v}_$rep.err; exit 1; }
    echo "prequeue=$v $rep $(python3 -c "import json; d=json.load(open('$out/sc_${v}_$rep.json')); print({k: (v['ms'], v['kernel_ms'], v['hbm_frac']) for k, v in d.items()})")"
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 tools/sc_bench.py 20,24 > $out/trace.log 2>&1 || exit 1
for rep in 1 2; do
  for c in default 19; do
    if [ $c = default ]; then e=TNS_AB_DEFAULT=1; else e=TNS_TABLE_C=$c; fi
    env $e timeout -k 10 200 python3 tools/c2c3_bench.py > $out/c2c3_${c}_$rep.json 2>&1 || { tail $out/c2c3_${c}_$rep.json; exit 1; }
    echo "table $c: $(cat $out/c2c3_${c}_$rep.json)"
  done
  for c in default 15; do
    if [ $c = default ]; then e=TNS_AB_DEFAULT=1; else e=TNS_TABLE_C=$c; fi
    env $e timeout -k 10 100 python3 tools/msm_trace.py 16 50 14 > $out/m16_${c}_$rep.txt 2>&1 || { tail $out/m16_${c}_$rep.txt; exit 1; }
    echo "table $c: $(tail -n 1 $out/m16_${c}_$rep.txt)"
  done
done
timeout -k 10 1500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $out/pytest_gpu.txt 2>&1 || { tail -30 $out/pytest_gpu.txt; exit 1; }
tail -2 $out/pytest_gpu.txt
