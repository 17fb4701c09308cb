#!/bin/bash
# opening-pair tail scheduling A/B: both tails after both accumulations (default for table-window
# pairs) vs lane 0's tail under lane 1's accumulation (TNS_TAILS_LAST=0).  tools/ab/ab_tails.sh
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "msm or MSM or lagrange or twist or shout or sharded" > gpurun_out/tails_pytest.log 2>&1
tail -2 gpurun_out/tails_pytest.log
bash tools/ab/ab_env.sh "TNS_NONE=0" "TNS_TAILS_LAST=0" "TNS_NONE=0" "TNS_TAILS_LAST=0" "TNS_TAILS_LAST=1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tails_ks -o run --output-format csv -- python3 bench.py --no-extras --steps 2 --warmup 1 > gpurun_out/tails_ks.log 2>&1
python3 tools/trace_tail.py gpurun_out/tails_ks/run_kernel_trace.csv k_u64_tables 0.03 > gpurun_out/tails_tail.txt
