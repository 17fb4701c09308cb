#!/bin/bash
# run one gpurun call, waiting (not retrying a failed run) while the pool has no free box (exit 3)
#   tools/gpurun_wait.sh <log> <timeout_s> '<command>'
log=$1; to=$2; cmd=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $log 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  grep -q "no free box\|slot(s) on this pod are busy\|retry in" $log || exit $rc
  sleep 90
done
exit 3
