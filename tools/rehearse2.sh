#!/bin/bash
# 2-rank sharded-proof rehearsal of bench.py on one GPU (gloo exchange, both ranks on device 0):
# one 2^25-op proof over 2 ranks.  tools/rehearse2.sh <tag>
set -euo pipefail
tag=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --rehearse-one-gpu > gpurun_out/rehearse_$tag.jsonl 2> gpurun_out/rehearse_$tag.err
tail -1 gpurun_out/rehearse_$tag.jsonl | cut -c1-400
