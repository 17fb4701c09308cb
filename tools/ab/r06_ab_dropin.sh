#!/bin/bash
# round 6: resident and drop-in C4 rates (extras trimmed), default library vs build variants,
# alternating on one box, then the 4-rank one-GPU rehearsal of each variant
#   tools/ab/r06_ab_dropin.sh <reps> <tag>...
set -uo pipefail
reps=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/multilinear-map-cryptography_amd
out=gpurun_out/r06_ab_dropin${AB_SUFFIX:-}
mkdir -p $out
for rep in $(seq 1 $reps); do
  for v in default "$@"; do
    if [ $v = default ]; then lib=$L/libtns.so; else lib=$L/libtns_$v.so; fi
    TNS_LIB=$lib timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --coef-steps 0 --tau-free-log 0 --sumcheck-logs "" \
      --c5-steps 0 --no-table-steps 0 --cpu-ref-logs 4-4 --cpu-fast-log-ops 14 > $out/b_${v}_$rep.jsonl 2> $out/b_${v}_$rep.err || { tail -5 $out/b_${v}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$out/b_${v}_$rep.jsonl').read().strip().splitlines()[-1])
print('$v rep $rep: resident', d['ms_per_step'], 'dropin', d.get('ms_per_step_dropin'), 'C2', d.get('msm_ms_2^20'))" | tee -a $out/summary.txt
  done
done
port=29571
for v in "$@"; do
  TNS_LIB=$L/libtns_$v.so timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 4 --steps 3 --warmup 1 --rehearse-one-gpu > $out/rehearse4_$v.jsonl 2> $out/rehearse4_$v.err || { tail -20 $out/rehearse4_$v.err; exit 1; }
  port=$((port + 1))
  python3 -c "
import json; r=json.loads(open('$out/rehearse4_$v.jsonl').read().strip().splitlines()[-1])
print('$v rehearse4', r['ms_per_step'], [round(p['mean_exchange_us']) for p in r['comm']['per_rank']])" | tee -a $out/summary.txt
done
