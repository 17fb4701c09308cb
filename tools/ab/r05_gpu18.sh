#!/bin/bash
# round 5 GPU pass 18: 6144-entry pass-1 tiles (three blocks per CU) vs 8192 -- MSM parity, C4 + C2 A/B
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu18
mkdir -p $out
TNS_BS_TILES=6144 timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "msm or twist or shout" > $out/pytest_t6144.txt 2>&1 || { tail -30 $out/pytest_t6144.txt; exit 1; }
tail -1 $out/pytest_t6144.txt
for rep in 1 2 3; do
  for v in 0 6144; do
    TNS_BS_TILES=$v timeout -k 10 200 python3 -u bench.py --no-extras --steps 10 --warmup 3 > $out/c4_t${v}_$rep.jsonl 2> $out/c4_t${v}_$rep.err || exit 1
    TNS_BS_TILES=$v timeout -k 10 100 python3 tools/msm_trace.py 20 20 18 > $out/c2_t${v}_$rep.txt 2>&1 || exit 1
    echo "tiles=$v rep $rep $(python3 -c "import json; d=json.loads(open('$out/c4_t${v}_$rep.jsonl').read().strip().splitlines()[-1]); s=d['stages_ms_per_step']; print(d['ms_per_step'], s.get('msm_sort'), s.get('msm_accumulate'), (d['device_state']['valu_clock_after_steps'] or {}).get('median_mhz'))") C2: $(tail -n 1 $out/c2_t${v}_$rep.txt)"
  done
done
bash tools/c4_step_trace.sh t6144 TNS_BS_TILES=6144 || exit 1
