#!/bin/bash
# pass-1 tile A/B: variant parity tests, C4 bench lines and standalone 2^20 / 2^24 MSMs with
# 8192- (default) and 4096-entry pass-1 tiles.  tools/ab/ab_p1tile.sh
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "bucket_sort_variants" > gpurun_out/p1tile_pytest.log 2>&1
tail -2 gpurun_out/p1tile_pytest.log
bash tools/ab/ab_env.sh "TNS_NONE=0" "TNS_BS_TILES=4096,8192,4096" "TNS_NONE=0" "TNS_BS_TILES=4096,8192,4096"
for e in "TNS_NONE=0" "TNS_BS_TILES=4096,8192,4096"; do
  for k in 20 24; do env $e timeout -k 10 120 python -u tools/msm_trace.py $k 10 | sed "s/^/$e /"; done
done
