#!/bin/bash
# the df7fe42 root-cause runs (tools/df7_check.py) for each staged build variant
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/df7
for v in "$@"; do
  for k in 18 20; do
    TNS_ICP_CHECK=1 timeout -k 10 120 python -u tools/df7_check.py tools/df7/$v $k >> gpurun_out/df7/check.txt 2>&1 || { echo "rc=$? for $v $k"; break 2; }
  done
done
cat gpurun_out/df7/check.txt
