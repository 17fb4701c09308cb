#!/bin/bash
# round 6: GPU suite, then the C4 bench at the driver's steps and a one-step kernel timeline:
#   tools/ab/r06_gpu.sh <tag> [skip-tests]
set -uo pipefail
tag=$1; skip=${2:-}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06_$tag
mkdir -p $out
if [ -z "$skip" ]; then
  timeout -k 10 1100 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $out/pytest_gpu.txt 2>&1 || { tail -30 $out/pytest_gpu.txt; exit 1; }
  tail -2 $out/pytest_gpu.txt
fi
timeout -k 10 200 python3 -u bench.py --no-extras --steps 20 --warmup 5 > $out/bench_c4.jsonl 2> $out/bench_c4.err || { tail -20 $out/bench_c4.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$out/bench_c4.jsonl').read().strip().splitlines()[-1]); s=d['stages_ms_per_step']
print('C4', d['ms_per_step'], 'acc', d['roofline']['avg_launch_ms'], {k: s[k] for k in sorted(s)})"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/tr -o run --output-format csv -- python3 bench.py --no-extras --steps 2 --warmup 1 > $out/trace_run.log 2>&1 || exit 1
f=$(find $out/tr -name "run_kernel_trace.csv" | head -n 1)
python3 tools/trace_tail.py "$f" k_u64_tables 0.05 > $out/timeline.txt 2>&1
tail -n 45 $out/timeline.txt | head -n 20
