set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/split
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/split/pytest.log 2>&1; tail -2 gpurun_out/split/pytest.log
bash tools/ab/ab_env.sh TNS_ACC_SPLIT=0 X=1 TNS_ACC_SPLIT=0.85 TNS_ACC_SPLIT=0 X=2
TNS_ACC_SPLIT=0 timeout -k 10 120 python3 -u tools/c2_tablec.py 20
timeout -k 10 120 python3 -u tools/c2_tablec.py 20
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/split/ks -o run --output-format csv -- python3 bench.py --no-extras --steps 2 --warmup 1 > gpurun_out/split/ks.log 2>&1
