#!/bin/bash
# round 4: C4 bench A/B over environment settings, alternating: tools/ab/r04_ab_env.sh <reps> "VAR=a" "VAR=b" ...
set -uo pipefail
reps=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04_abenv
mkdir -p $out
for rep in $(seq 1 $reps); do
  for v in "$@"; do
    tag=$(echo "$v" | tr ' =' '__')
    env $v timeout -k 10 200 python3 -u bench.py --no-extras --steps 10 --warmup 3 > $out/c4_${tag}_$rep.jsonl 2> $out/c4_${tag}_$rep.err || exit $?
    echo "$v rep $rep C4: $(python3 -c "import json; d=json.loads(open('$out/c4_${tag}_$rep.jsonl').read().strip().splitlines()[-1]); s=d['stages_ms_per_step']; print(d['ms_per_step'], d['roofline']['avg_launch_ms'], s['msm_accumulate'], s['msm_fixup'], s['msm_reduce'])")"
  done
done
