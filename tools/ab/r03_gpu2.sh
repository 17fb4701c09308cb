#!/bin/bash
# round-3 GPU pass on the current tree: the GPU parity suite, the driver-style bench line,
# and a rocprofv3 kernel-stats pass of the same bench command
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${OUT:-r03g2}
mkdir -p $out
if [ "${SKIP_TESTS:-0}" = 0 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:-} > $out/pytest_gpu.log 2>&1
  rc=$?
  tail -5 $out/pytest_gpu.log
  [ $rc = 0 ] || exit $rc
fi
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $out/bench.jsonl 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc = 0 ] || { tail -20 $out/bench.err; exit $rc; }
tail -c 3000 $out/bench.jsonl
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 -u bench.py --steps 20 --warmup 5 --no-extras > $out/bench_prof.jsonl 2> $out/bench_prof.err
  rc=$?; echo "prof rc=$rc"; [ $rc = 0 ] || exit $rc
  find $out/prof -name "*kernel_stats.csv" | head -3
fi
