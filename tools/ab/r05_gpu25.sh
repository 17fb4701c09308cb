#!/bin/bash
# round 5 GPU pass 25: a 10-bit last sort pass (TNS_BS_BITS 8,7,10 / 7,8,10 for the 25-bit opening keys,
# 7,6,10 / 6,7,10 for C2's 23-bit keys) -- parity under each, C4 + C2 A/B vs the default split
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu25
mkdir -p $out
for b in 8,7,10 7,6,10; do
  TNS_BS_BITS=$b timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py -k "msm or twist or shout or c2 or c4" > $out/pytest_$b.txt 2>&1 || { tail -30 $out/pytest_$b.txt; exit 1; }
  echo "TNS_BS_BITS=$b $(tail -1 $out/pytest_$b.txt)"
done
for rep in 1 2 3; do
  for b in default 8,7,10 7,8,10; do
    if [ $b = default ]; then e=TNS_AB_DEFAULT=1; else e=TNS_BS_BITS=$b; fi
    env $e timeout -k 10 200 python3 -u bench.py --no-extras --steps 10 --warmup 3 > $out/c4_${b}_$rep.jsonl 2> $out/c4_${b}_$rep.err || exit 1
    echo "C4 $b rep $rep $(python3 -c "import json; d=json.loads(open('$out/c4_${b}_$rep.jsonl').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['stages_ms_per_step'].get('msm_sort'))")"
  done
  for b in default 7,6,10 6,7,10; do
    if [ $b = default ]; then e=TNS_AB_DEFAULT=1; else e=TNS_BS_BITS=$b; fi
    env $e timeout -k 10 100 python3 tools/msm_trace.py 20 50 18 > $out/c2_${b}_$rep.txt 2>&1 || exit 1
    echo "C2 $b rep $rep $(tail -n 1 $out/c2_${b}_$rep.txt)"
  done
done
bash tools/c4_step_trace.sh bits8710 TNS_BS_BITS=8,7,10 || exit 1
