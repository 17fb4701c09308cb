#!/bin/bash
# standalone 2^k MSM kernel traces under env settings: tools/ab/ab_msm_env.sh <tag> <log_n> "VAR=a VAR2=b" ...
# prints the per-kernel durations of the last MSM of each setting
set -euo pipefail
tag=$1; k=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
i=0
for e in "$@"; do
  d=gpurun_out/abm_${tag}_$i
  env $e timeout -k 10 240 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python3 tools/msm_trace.py $k 2 > $d.log 2>&1
  echo "== $e: $(tail -1 $d.log)"
  python3 tools/last_msm.py $(find $d -name "*kernel_trace.csv" | head -1)
  i=$((i+1))
done
