#!/bin/bash
# C2 (2^20 full-width MSM) reduction-shape A/B: tools/ab/ab_c2red.sh "VAR=a VAR2=b" ...
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for rep in 1 2; do
  for e in "$@"; do
    env $e timeout -k 10 120 python -u tools/msm_trace.py 20 30 | sed "s/^/[$e] /"
  done
done
