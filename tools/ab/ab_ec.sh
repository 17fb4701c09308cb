#!/bin/bash
# A/B on one box: the C4 bench with the early-clobber-free asm (libtns.so) vs the old asm (libtns_oldasm.so)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab_ec
for i in 1 2; do
  for t in lib oldasm; do
    if [ $t = lib ]; then lib=$PWD/multilinear-map-cryptography_amd/libtns.so; else lib=$PWD/multilinear-map-cryptography_amd/libtns_$t.so; fi
    TNS_LIB=$lib timeout -k 10 200 python -u bench.py --no-extras --steps 20 --warmup 5 > gpurun_out/ab_ec/$t$i.jsonl 2>gpurun_out/ab_ec/$t$i.err || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/ab_ec/$t$i.jsonl').read().strip().splitlines()[-1]);print('$t', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done
