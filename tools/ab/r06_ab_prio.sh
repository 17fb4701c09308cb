#!/bin/bash
# round 6: stream priorities (TNS_STREAM_PRIO build variants: default = context high / lane 1 normal /
# accumulations low, pa = context normal / lane 1 low / accumulations low, pb = all normal):
# C4 A/B, then the 4-rank one-GPU rehearsal per variant
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/multilinear-map-cryptography_amd
out=gpurun_out/r06_ab_prio
mkdir -p $out
bash tools/ab/r06_ab_lib.sh prio 4 "$@" || exit 1
port=29561
for v in default "$@"; do
  if [ $v = default ]; then lib=$L/libtns.so; else lib=$L/libtns_$v.so; fi
  TNS_LIB=$lib timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 4 --steps 3 --warmup 1 --rehearse-one-gpu > $out/rehearse4_$v.jsonl 2> $out/rehearse4_$v.err || { tail -20 $out/rehearse4_$v.err; exit 1; }
  port=$((port + 1))
  python3 -c "
import json; r=json.loads(open('$out/rehearse4_$v.jsonl').read().strip().splitlines()[-1])
print('$v rehearse4', r['ms_per_step'], [round(p['mean_exchange_us']) for p in r['comm']['per_rank']])" | tee -a $out/summary.txt
done
