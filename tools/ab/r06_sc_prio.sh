#!/bin/bash
# round 6: the generic sum-check (2^20, 2^24) with the context stream at the greatest priority
# (default) vs a context without stream priorities, alternating
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06_sc_prio
mkdir -p $out
for rep in 1 2 3; do
  for v in prio noprio; do
    for k in 20 24; do
      timeout -k 10 120 python3 tools/sc_trace.py $k 30 $v > $out/${v}_${k}_$rep.txt 2>&1 || { cat $out/${v}_${k}_$rep.txt; exit 1; }
      echo "$v rep $rep $(cat $out/${v}_${k}_$rep.txt)" | tee -a $out/summary.txt
    done
  done
done
