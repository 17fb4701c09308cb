#!/bin/bash
# round-3 A/B: selected GPU tests, then the C4 bench with each env setting in $AB (";"-separated,
# "-" = defaults), alternating twice; prints ms/step, the accumulate average and the stage sums
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${OUT:-r03ab}
mkdir -p $out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$TESTS" > $out/pytest.log 2>&1
  rc=$?; tail -3 $out/pytest.log; [ $rc = 0 ] || { grep -E "Error|assert|FAILED" $out/pytest.log | head -20; exit $rc; }
fi
IFS=';' read -ra VARS <<< "${AB:--}"
for rep in 1 2; do
  for v in "${VARS[@]}"; do
    tag=$(echo "$v" | tr -c 'A-Za-z0-9_=\n' '_')
    ( [ "$v" != "-" ] && export $v; timeout -k 10 200 python -u bench.py --no-extras --steps ${STEPS:-10} --warmup 3 > $out/b_${tag}_$rep.jsonl 2> $out/b_${tag}_$rep.err )
    rc=$?; [ $rc = 0 ] || { echo "bench $v rc=$rc"; tail -5 $out/b_${tag}_$rep.err; exit $rc; }
    python3 -c "
import json,sys
d=json.loads(open('$out/b_${tag}_$rep.jsonl').read().strip().splitlines()[-1])
print('%-40s %8.3f ms/step  acc %.3f  stages %s' % ('$v', d['ms_per_step'], d['roofline']['avg_launch_ms'], {k: round(x, 2) for k, x in d['stages_ms_per_step'].items()}))"
  done
done
