#!/bin/bash
# 4-rank sharded-proof rehearsal of bench.py on one GPU (gloo exchange, every rank on device 0):
# one 2^26-op proof over 4 ranks (the N = 4 code path: two folded rounds on the host).  tools/rehearse4.sh <tag>
set -euo pipefail
tag=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29534 bench.py --gpus 4 --steps 2 --warmup 1 --rehearse-one-gpu > gpurun_out/rehearse4_$tag.jsonl 2> gpurun_out/rehearse4_$tag.err
tail -1 gpurun_out/rehearse4_$tag.jsonl | cut -c1-600
