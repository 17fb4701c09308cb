#!/bin/bash
# C4 bench under several environment settings: tools/ab/ab_env.sh "VAR=a" "VAR=b" ...
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
i=0
for e in "$@"; do
  env $e timeout -k 10 200 python -u bench.py --no-extras --steps 8 > gpurun_out/ab$i.jsonl 2>gpurun_out/ab$i.err
  python3 -c "
import json,sys
d=json.load(open('gpurun_out/ab$i.jsonl')); print('$e', d['ms_per_step'], d['twist_last_prove_ms']['open'], d['stages_ms_per_step'])"
  i=$((i+1))
done
