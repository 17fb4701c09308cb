#!/bin/bash
# A/B of library builds with kernel traces: tools/ab/ab_lib_ks.sh <log_n> <tag>...  (tag "lib" = libtns.so,
# else multilinear-map-cryptography_amd/libtns_<tag>.so): the last standalone 2^log_n MSM's kernels, then
# one C4 bench line (ms/step and per-stage device time) per build
set -euo pipefail
k=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for t in "$@"; do
  if [ "$t" = lib ]; then lib=$PWD/multilinear-map-cryptography_amd/libtns.so; else lib=$PWD/multilinear-map-cryptography_amd/libtns_$t.so; fi
  d=gpurun_out/abk_$t
  TNS_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python3 tools/msm_trace.py $k 2 > $d.log 2>&1
  echo "== $t: $(tail -1 $d.log)"
  python3 tools/last_msm.py $(find $d -name "*kernel_trace.csv" | head -1)
  TNS_LIB=$lib timeout -k 10 200 python -u bench.py --no-extras --steps 8 > gpurun_out/ab_$t.jsonl 2>gpurun_out/ab_$t.err
  python3 -c "
import json
d=json.load(open('gpurun_out/ab_$t.jsonl')); print('  $t C4', d['ms_per_step'], d['stages_ms_per_step'])"
done
