#!/bin/bash
# GPU tests, then the C4 bench with the rocPRIM digit sort vs bucket_sort_dev, then a kernel trace.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1 || { tail -30 gpurun_out/pt.log; exit 1; }
tail -2 gpurun_out/pt.log
TNS_MSM_SORT=cub timeout -k 10 200 python -u bench.py --no-extras --steps 4 > gpurun_out/abc.jsonl 2>gpurun_out/abc.err
timeout -k 10 200 python -u bench.py --no-extras --steps 4 > gpurun_out/abn.jsonl 2>gpurun_out/abn.err
python3 -c "
import json
for f in ['abc','abn']:
    d=json.load(open('gpurun_out/%s.jsonl'%f)); print(f, d['ms_per_step'], d['twist_last_prove_ms'], d['stages_ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ks -o run --output-format csv -- python3 bench.py --no-extras --steps 2 --warmup 1 > gpurun_out/ks.log 2>&1
