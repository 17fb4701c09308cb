#!/bin/bash
# round 5: C4 bench (no extras) under environment settings, alternating on one box:
#   tools/ab/r05_ab_env.sh <name> <reps> "VAR=a" "VAR=b" ...   ("-" = the default environment)
set -uo pipefail
name=$1; reps=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_abenv_$name
mkdir -p $out
for rep in $(seq 1 $reps); do
  i=0
  for e in "$@"; do
    if [ "$e" = "-" ]; then e=TNS_AB_DEFAULT=1; fi
    env $e timeout -k 10 200 python3 -u bench.py --no-extras --steps 10 --warmup 3 > $out/c4_${i}_$rep.jsonl 2> $out/c4_${i}_$rep.err || exit $?
    echo "$e rep $rep: $(python3 -c "
import json; d=json.loads(open('$out/c4_${i}_$rep.jsonl').read().strip().splitlines()[-1]); s=d['stages_ms_per_step']; t=d['twist_last_prove_ms']
print(d['ms_per_step'], 'commit', t.get('commit'), 'open', t.get('open'), 'sort', s.get('msm_sort'), 'acc', s.get('msm_accumulate'), 'fix', s.get('msm_fixup'), 'red', s.get('msm_reduce'), 'clk', (d['device_state']['valu_clock_after_steps'] or {}).get('median_mhz'))")"
    i=$((i+1))
  done
done
