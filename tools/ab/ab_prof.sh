#!/bin/bash
# timed-region profiling A/B: only the roofline kernel timed (default) vs every stage timed
# inside the timed steps (--profile-all-timed).  tools/ab/ab_prof.sh
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
i=0
for a in "" "--profile-all-timed" "" "--profile-all-timed"; do
  timeout -k 10 200 python -u bench.py --no-extras --steps 10 --warmup 2 $a > gpurun_out/abp$i.jsonl 2>gpurun_out/abp$i.err
  python3 -c "
import json
d=json.load(open('gpurun_out/abp$i.jsonl')); print('[$a]', d['ms_per_step'], d['twist_last_prove_ms']['total'], d['roofline']['avg_launch_ms'], d['stages_ms_per_step'].get('msm_accumulate'), d.get('stages_timed_on'))"
  i=$((i+1))
done
