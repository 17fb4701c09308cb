#!/bin/bash
# round 5 GPU pass 22: MSM host readbacks through mapped memory + flag polling (default) vs pinned copies +
# stream synchronize (TNS_MSM_SYNC_READBACK=1) -- GPU suite, C2 and C4 A/B, C2 trace
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu22
mkdir -p $out
timeout -k 10 1500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $out/pytest_gpu.txt 2>&1 || { tail -30 $out/pytest_gpu.txt; exit 1; }
tail -2 $out/pytest_gpu.txt
for rep in 1 2 3; do
  for v in 0 1; do
    TNS_MSM_SYNC_READBACK=$v timeout -k 10 100 python3 tools/msm_trace.py 20 50 18 > $out/c2_s${v}_$rep.txt 2>&1 || exit 1
    TNS_MSM_SYNC_READBACK=$v timeout -k 10 200 python3 -u bench.py --no-extras --steps 10 --warmup 3 > $out/c4_s${v}_$rep.jsonl 2> $out/c4_s${v}_$rep.err || exit 1
    echo "sync_readback=$v rep $rep C4 $(python3 -c "import json; d=json.loads(open('$out/c4_s${v}_$rep.jsonl').read().strip().splitlines()[-1]); print(d['ms_per_step'])") C2: $(tail -n 1 $out/c2_s${v}_$rep.txt)"
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/c2_trace -o run --output-format csv -- python3 tools/msm_trace.py 20 20 18 > $out/c2_trace.log 2>&1 || exit 1
