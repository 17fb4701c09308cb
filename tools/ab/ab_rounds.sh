#!/bin/bash
# accumulation chunk sizing A/B: round-filling chunks (default) vs the power-of-two rule
# (TNS_ACC_ROUNDS=0): MSM/sort parity tests, C4 bench lines, standalone 2^20 / 2^24 MSMs.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "msm or MSM or sort or lagrange or twist or shout or sharded" > gpurun_out/rounds_pytest.log 2>&1
tail -2 gpurun_out/rounds_pytest.log
bash tools/ab/ab_env.sh "TNS_NONE=0" "TNS_ACC_ROUNDS=0" "TNS_NONE=0" "TNS_ACC_ROUNDS=0"
for e in "TNS_NONE=0" "TNS_ACC_ROUNDS=0" "TNS_NONE=0" "TNS_ACC_ROUNDS=0"; do
  env $e timeout -k 10 120 python -u tools/msm_trace.py 20 20 | sed "s/^/$e /"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rounds_ks -o run --output-format csv -- python3 bench.py --no-extras --steps 2 --warmup 1 > gpurun_out/rounds_ks.log 2>&1
python3 tools/trace_tail.py gpurun_out/rounds_ks/run_kernel_trace.csv k_u64_tables 0.03 > gpurun_out/rounds_tail.txt
bash tools/ab/msm_ks.sh rnd20 20
python3 tools/trace_tail.py gpurun_out/msm_rnd20/run_kernel_trace.csv k_scalar_bits > gpurun_out/msm_rnd20_tail.txt
