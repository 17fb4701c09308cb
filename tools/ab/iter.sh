#!/bin/bash
# One iteration on the GPU: MSM/sort parity tests, standalone MSM traces (2^24, 2^20) and
# C4 bench lines under env settings.  tools/ab/iter.sh <tag> [ENV=val ...]  (each env = one bench line)
set -euo pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "msm or MSM or lagrange or twist or shout or sharded" > gpurun_out/it_$tag.pytest 2>&1
tail -2 gpurun_out/it_$tag.pytest
tools/ab/msm_ks.sh ${tag}24 24
tools/ab/msm_ks.sh ${tag}20 20
i=0
for e in "$@"; do
  env $e timeout -k 10 200 python -u bench.py --steps 8 > gpurun_out/it_${tag}_$i.jsonl 2>gpurun_out/it_${tag}_$i.err
  python3 -c "
import json
d=json.load(open('gpurun_out/it_${tag}_$i.jsonl')); print('$e', d['ms_per_step'], d['twist_last_prove_ms'], d['stages_ms_per_step'], d.get('msm_pairs_per_sec_2^20'))"
  i=$((i+1))
done
