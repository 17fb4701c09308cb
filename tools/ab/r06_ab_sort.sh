#!/bin/bash
# round 6: same-box A/B of HEAD, the round-5 evidence tree cfc4505 (ab6/cfc) and HEAD with the three
# last sort commits 0f561b1/7d8c4f0/bff3282 reverted (ab6/rev); C4 at the driver's steps, alternating:
#   tools/ab/r06_ab_sort.sh [reps]
set -uo pipefail
reps=${1:-3}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06_ab_sort
mkdir -p $out
for rep in $(seq 1 $reps); do
  for v in head cfc rev; do
    if [ $v = head ]; then d=.; else d=ab6/$v; fi
    (cd $d && timeout -k 10 200 python3 -u bench.py --no-extras --gpus 1 --steps 20 --warmup 5) > $out/${v}_$rep.jsonl 2> $out/${v}_$rep.err || exit $?
    echo "$v rep $rep: $(python3 -c "
import json; d=json.loads(open('$out/${v}_$rep.jsonl').read().strip().splitlines()[-1])
s=d['stages_ms_per_step']; ds=d.get('device_state') or {}
print('step', d['ms_per_step'], 'acc', d['roofline']['avg_launch_ms'], 'sort', s.get('msm_sort'), 'accst', s.get('msm_accumulate'), 'mhz', (ds.get('valu_clock_after_steps') or {}).get('median_mhz'))")" | tee -a $out/summary.txt
  done
done
