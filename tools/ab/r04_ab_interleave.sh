#!/bin/bash
# round 4: TNS_SORT_INTERLEAVE=1 (both lanes' pass 1 queued before either lane's later passes) A/B
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04_il
mkdir -p $out
for rep in 1 2 3; do
  for v in "TNS_SORT_INTERLEAVE=0" "TNS_SORT_INTERLEAVE=1"; do
    env $v timeout -k 10 200 python3 -u bench.py --no-extras --steps 10 --warmup 3 > $out/c4_${v}_$rep.jsonl 2> $out/c4_${v}_$rep.err || exit $?
    echo "$v rep $rep C4: $(python3 -c "import json; d=json.loads(open('$out/c4_${v}_$rep.jsonl').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['twist_last_prove_ms'])")"
  done
done
