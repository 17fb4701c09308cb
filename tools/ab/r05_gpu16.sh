#!/bin/bash
# round 5 GPU pass 16: persistent tail range x block-count sweep
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu16
mkdir -p $out
for rep in 1 2; do
  for v in "13 64" "13 32" "13 16" "12 32" "14 32" "15 64" "16 64" "15 128"; do
    set -- $v
    TNS_SC_TAIL_LOG=$1 TNS_SC_TAIL_BLOCKS=$2 timeout -k 10 200 python3 -u tools/sc_bench.py 20,24 > $out/sc_$1_$2_$rep.json 2> $out/sc_$1_$2_$rep.err || { cat $out/sc_$1_$2_$rep.err; exit 1; }
    echo "tail<=2^$1 blocks<=$2 $rep $(python3 -c "import json; d=json.load(open('$out/sc_$1_$2_$rep.json')); print({k: (v['ms'], v['kernel_ms'], v['hbm_frac']) for k, v in d.items()})")"
  done
done
