#!/bin/bash
# A/B of library builds on the GPU box: tools/ab/ab_lib.sh <log_n> <tag>...  (tag "lib" = libtns.so,
# else multilinear-map-cryptography_amd/libtns_<tag>.so); standalone MSM 2^log_n then one C4 bench line each
set -euo pipefail
k=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for t in "$@"; do
  if [ "$t" = lib ]; then lib=$PWD/multilinear-map-cryptography_amd/libtns.so; else lib=$PWD/multilinear-map-cryptography_amd/libtns_$t.so; fi
  echo -n "$t: "; TNS_LIB=$lib timeout -k 10 120 python -u tools/msm_trace.py $k 6 2>&1 | tail -1
  TNS_LIB=$lib timeout -k 10 200 python -u bench.py --no-extras --steps 8 > gpurun_out/ab_$t.jsonl 2>gpurun_out/ab_$t.err
  python3 -c "
import json
d=json.load(open('gpurun_out/ab_$t.jsonl')); print('  $t C4', d['ms_per_step'], d['stages_ms_per_step'])"
done
