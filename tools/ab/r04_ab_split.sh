#!/bin/bash
# round 4: drop-in value chunks with the last chunk split in two (default) vs four equal chunks
# (TNS_UPLOAD_SPLIT_LAST=0), and TNS_SORT_INTERLEAVE A/B on the resident C4 step
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04_split
mkdir -p $out
for rep in 1 2; do
  for v in "TNS_UPLOAD_SPLIT_LAST=1" "TNS_UPLOAD_SPLIT_LAST=0"; do
    env $v timeout -k 10 120 python3 tools/dropin_trace.py 22 6 > $out/di_${v}_$rep.txt 2>&1 || exit $?
    echo "$v rep $rep: $(grep '^dropin' $out/di_${v}_$rep.txt | cut -c1-60)"
  done
  for v in "TNS_SORT_INTERLEAVE=0" "TNS_SORT_INTERLEAVE=1"; do
    env $v timeout -k 10 200 python3 -u bench.py --no-extras --steps 10 --warmup 3 > $out/c4_${v}_$rep.jsonl 2> $out/c4_${v}_$rep.err || exit $?
    echo "$v rep $rep C4: $(python3 -c "import json; d=json.loads(open('$out/c4_${v}_$rep.jsonl').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['twist_last_prove_ms'])")"
  done
done
