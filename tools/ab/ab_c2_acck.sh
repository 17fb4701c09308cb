#!/bin/bash
# C2 (2^20 MSM) per accumulation chunk size: tools/ab/ab_c2_acck.sh 32 64 70 ...
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for k in "$@"; do
  echo -n "TNS_ACC_K=$k "; TNS_ACC_K=$k timeout -k 10 120 python3 tools/c2_tablec.py 20 | tail -1
done
echo -n "default "; timeout -k 10 120 python3 tools/c2_tablec.py 20 | tail -1
