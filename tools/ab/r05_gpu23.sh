#!/bin/bash
# round 5 GPU pass 23: one-launch sort geometry (k_bs_geom) -- GPU suite, C2 / C4 A/B vs TNS_BS_GEOM=0, C2 trace
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu23
mkdir -p $out
timeout -k 10 1500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $out/pytest_gpu.txt 2>&1 || { tail -30 $out/pytest_gpu.txt; exit 1; }
tail -2 $out/pytest_gpu.txt
for rep in 1 2 3; do
  for v in 1 0; do
    TNS_BS_GEOM=$v timeout -k 10 100 python3 tools/msm_trace.py 20 50 18 > $out/c2_g${v}_$rep.txt 2>&1 || exit 1
    TNS_BS_GEOM=$v timeout -k 10 200 python3 -u bench.py --no-extras --steps 10 --warmup 3 > $out/c4_g${v}_$rep.jsonl 2> $out/c4_g${v}_$rep.err || exit 1
    echo "geom=$v rep $rep C4 $(python3 -c "import json; d=json.loads(open('$out/c4_g${v}_$rep.jsonl').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['stages_ms_per_step'].get('msm_sort'))") C2: $(tail -n 1 $out/c2_g${v}_$rep.txt)"
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/c2_trace -o run --output-format csv -- python3 tools/msm_trace.py 20 20 18 > $out/c2_trace.log 2>&1 || exit 1
