#!/bin/bash
# round 5 GPU pass 2: sum-check parity tests on the new round kernel, its bench numbers, then the
# evidence pass (tools/ab/r05_prof1.sh).
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu2
mkdir -p $out
timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0, 'multilinear-map-cryptography_amd')
import twist_and_shout as ts
ctx = ts.Context.get(0)
print('clock probe', ts.clock_probe(ctx, 60.0), ts.clock_probe(ctx, 200.0), flush=True)" > $out/clock.txt 2>&1 || { cat $out/clock.txt; exit 1; }
cat $out/clock.txt
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sumcheck.py tests/test_gpu_parity.py -k "sumcheck" > $out/pytest_sc.txt 2>&1 || { tail -30 $out/pytest_sc.txt; exit 1; }
tail -2 $out/pytest_sc.txt
timeout -k 10 200 python3 -u tools/sc_bench.py 20,24 > $out/sc_bench.json 2> $out/sc_bench.err || { cat $out/sc_bench.err; exit 1; }
cat $out/sc_bench.json
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/sc_trace -o run --output-format csv -- python3 tools/sc_bench.py 20 > $out/sc_trace.log 2>&1 || exit 1
bash tools/ab/r05_prof1.sh || exit 1
timeout -k 10 900 bash tools/ab/r05_ab_libs.sh bsblock 2 bs512 bs1024
