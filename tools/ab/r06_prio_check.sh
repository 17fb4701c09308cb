#!/bin/bash
# round 6: the context-creation flag TNS_CTX_NO_STREAM_PRIORITIES: its GPU test, the C4 bench and
# the 2- / 4-rank one-GPU rehearsals (created without priorities)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06_prio_check
mkdir -p $out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_configs.py -k "stream_priorities or msm_tables_off" > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
timeout -k 10 200 python3 -u bench.py --no-extras --steps 20 --warmup 5 > $out/c4.jsonl 2> $out/c4.err || { tail -5 $out/c4.err; exit 1; }
tail -c 200 $out/c4.jsonl; echo
for n in 2 4; do
  timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29580 + n)) bench.py --gpus $n --steps 3 --warmup 1 --rehearse-one-gpu > $out/rehearse$n.jsonl 2> $out/rehearse$n.err || { tail -20 $out/rehearse$n.err; exit 1; }
  python3 -c "
import json; r=json.loads(open('$out/rehearse$n.jsonl').read().strip().splitlines()[-1])
print('rehearse$n', r['ms_per_step'], [round(p['mean_exchange_us']) for p in r['comm']['per_rank']])"
done
