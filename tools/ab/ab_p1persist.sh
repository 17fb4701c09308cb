#!/bin/bash
# persistent prefetching pass-1 scatter A/B: MSM/sort parity tests, C4 bench lines and standalone
# 2^20 / 2^24 MSMs with the persistent grid (default) and one block per tile (TNS_BS_P1_BLOCKS=0).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "msm or MSM or sort or lagrange or twist or shout" > gpurun_out/p1p_pytest.log 2>&1
tail -2 gpurun_out/p1p_pytest.log
bash tools/ab/ab_env.sh "TNS_NONE=0" "TNS_BS_P1_BLOCKS=0" "TNS_NONE=0" "TNS_BS_P1_BLOCKS=0"
for e in "TNS_NONE=0" "TNS_BS_P1_BLOCKS=0"; do
  for k in 20 24; do env $e timeout -k 10 120 python -u tools/msm_trace.py $k 10 | sed "s/^/$e /"; done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p1p_ks -o run --output-format csv -- python3 bench.py --no-extras --steps 2 --warmup 1 > gpurun_out/p1p_ks.log 2>&1
python3 tools/trace_tail.py gpurun_out/p1p_ks/run_kernel_trace.csv k_u64_tables 0.03 > gpurun_out/p1p_tail.txt
