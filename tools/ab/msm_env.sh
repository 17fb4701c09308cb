#!/bin/bash
# standalone MSM timing under env settings: tools/ab/msm_env.sh <log_n> "VAR=a" "VAR=b" ...
set -euo pipefail
k=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for e in "$@"; do
  echo -n "$e: "
  env $e timeout -k 10 120 python -u tools/msm_trace.py $k 6 2>&1 | tail -1
done
