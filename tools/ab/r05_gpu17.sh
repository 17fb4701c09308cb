#!/bin/bash
# round 5 GPU pass 17: defaults with the persistent tail -- full GPU suite, sum-check bench x2, smoke
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu17
mkdir -p $out
timeout -k 10 1500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $out/pytest_gpu.txt 2>&1 || { tail -30 $out/pytest_gpu.txt; exit 1; }
tail -2 $out/pytest_gpu.txt
for rep in 1 2; do
  timeout -k 10 200 python3 -u tools/sc_bench.py 20,24 > $out/sc_$rep.json 2> $out/sc_$rep.err || { cat $out/sc_$rep.err; exit 1; }
  cat $out/sc_$rep.json | cut -c1-600
done
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || { tail -20 $out/smoke.txt; exit 1; }
tail -3 $out/smoke.txt
