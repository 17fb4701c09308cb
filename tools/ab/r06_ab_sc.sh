#!/bin/bash
# round 6: generic sum-check schedule A/B (build variants libtns_<tag>.so), alternating on one box:
#   tools/ab/r06_ab_sc.sh <reps> <tag>...
set -uo pipefail
reps=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06_ab_sc
mkdir -p $out
L=$GRAFT_REPO_ROOT/multilinear-map-cryptography_amd
for rep in $(seq 1 $reps); do
  for v in default "$@"; do
    if [ $v = default ]; then lib=$L/libtns.so; else lib=$L/libtns_$v.so; fi
    for k in 20 24; do
      TNS_LIB=$lib timeout -k 10 120 python3 tools/sc_trace.py $k 20 > $out/${v}_${k}_$rep.txt 2>&1 || { cat $out/${v}_${k}_$rep.txt; exit 1; }
      echo "$v rep $rep $(cat $out/${v}_${k}_$rep.txt)" | tee -a $out/summary.txt
    done
  done
done
