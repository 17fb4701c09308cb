set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/w1; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "variants_agree" > $o/pytest.log 2>&1; tail -2 $o/pytest.log
timeout -k 10 200 python -u bench.py --no-extras > $o/b1.jsonl 2>&1; grep -o '"ms_per_step": [0-9.]*\|"twist_last_prove_ms": {[^}]*}' $o/b1.jsonl
TNS_MSM_W1=0 timeout -k 10 200 python -u bench.py --no-extras > $o/b0.jsonl 2>&1; grep -o '"ms_per_step": [0-9.]*\|"twist_last_prove_ms": {[^}]*}' $o/b0.jsonl
timeout -k 10 200 python -u bench.py --no-extras > $o/b1b.jsonl 2>&1; grep -o '"ms_per_step": [0-9.]*\|"twist_last_prove_ms": {[^}]*}' $o/b1b.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace -d $o/ks -o run --output-format csv -- python3 bench.py --no-extras --steps 2 --warmup 1 > $o/ks.log 2>&1
