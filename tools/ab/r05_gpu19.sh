#!/bin/bash
# round 5 GPU pass 19: C2 bucket-reduction shape sweep for the c = 20 table plan (2^19 buckets):
# first-level group L0 (TNS_RED_L), second level L1 (TNS_RED_L1), masked-sum chunk (TNS_RED_CH)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu19
mkdir -p $out
for rep in 1 2; do
  for l in 2 4 8; do for l1 in 0 2 4 8; do for ch in 4 8 16; do
    TNS_RED_L=$l TNS_RED_L1=$l1 TNS_RED_CH=$ch timeout -k 10 100 python3 tools/msm_trace.py 20 20 18 > $out/c2_${l}_${l1}_${ch}_$rep.txt 2>&1 || exit 1
    echo "L0=$l L1=$l1 CH=$ch rep $rep $(tail -n 1 $out/c2_${l}_${l1}_${ch}_$rep.txt)"
  done; done; done
  timeout -k 10 100 python3 tools/msm_trace.py 20 20 18 > $out/c2_default_$rep.txt 2>&1 || exit 1
  echo "default rep $rep $(tail -n 1 $out/c2_default_$rep.txt)"
done
