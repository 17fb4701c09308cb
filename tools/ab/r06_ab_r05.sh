#!/bin/bash
# round 6: same-box A/B of the closing tree (HEAD) and round 5's last tree abf9eac (worktree
# ab6/r05, its own bench.py and library), C4 at the driver's steps, alternating:
#   tools/ab/r06_ab_r05.sh [reps]
set -uo pipefail
reps=${1:-4}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06_ab_r05
mkdir -p $out
for rep in $(seq 1 $reps); do
  for v in head r05; do
    if [ $v = head ]; then d=.; else d=ab6/$v; fi
    (cd $d && timeout -k 10 200 python3 -u bench.py --no-extras --gpus 1 --steps 20 --warmup 5) > $out/${v}_$rep.jsonl 2> $out/${v}_$rep.err || exit $?
    echo "$v rep $rep: $(python3 -c "
import json; d=json.loads(open('$out/${v}_$rep.jsonl').read().strip().splitlines()[-1])
s=d['stages_ms_per_step']; t=d['twist_last_prove_ms']
print('step', d['ms_per_step'], 'commit', t['commit'], 'open', t['open'], 'acc', d['roofline']['avg_launch_ms'])")" | tee -a $out/summary.txt
  done
done
