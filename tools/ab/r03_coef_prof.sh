#!/bin/bash
# kernel stats of the coefficient route (interpolation + coefficient KZG) at C4
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${OUT:-r03coef}
mkdir -p $out
timeout -k 10 300 python -u bench.py --no-extras --commit-basis coefficients --steps 2 --warmup 1 > $out/bench.jsonl 2> $out/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc = 0 ] || { tail -5 $out/bench.err; exit $rc; }
python3 -c "
import json; d=json.loads(open('$out/bench.jsonl').read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('twist_last_prove_ms'), d['stages_ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 -u bench.py --no-extras --commit-basis coefficients --steps 2 --warmup 1 > $out/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc = 0 ] || exit $rc
find $out/prof -name "*kernel_stats.csv" | head -2
