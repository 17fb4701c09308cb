#!/bin/bash
# round-3 pass: full GPU suite on the current tree, coefficient-route kernel stats, drop-in trace
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${OUT:-r03g3}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; tail -3 $out/pytest_gpu.log; [ $rc = 0 ] || { grep -E "Error|assert|FAILED" $out/pytest_gpu.log | head; exit $rc; }
timeout -k 10 200 python -u tools/dropin_trace.py > $out/dropin.txt 2>&1
rc=$?; cat $out/dropin.txt; [ $rc = 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $out/di -o run --output-format csv -- python3 -u tools/dropin_trace.py 22 3 > $out/di.log 2>&1
rc=$?; echo "di trace rc=$rc"; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-extras --commit-basis coefficients --steps 2 --warmup 1 > $out/coef.jsonl 2> $out/coef.err
rc=$?; echo "coef rc=$rc"; [ $rc = 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/coefprof -o run --output-format csv -- python3 -u bench.py --no-extras --commit-basis coefficients --steps 2 --warmup 1 > $out/coefprof.log 2>&1
echo "coef prof rc=$?"
