#!/bin/bash
# round 5 closing evidence on the last tree: the bench as the driver runs it, its rocprofv3 cross-check,
# the 2-rank sharded rehearsal on one GPU
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_final4
mkdir -p $out
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.jsonl 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
tail -n 1 $out/bench.jsonl | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-extras > $out/prof_bench.jsonl 2> $out/prof_bench.err || { tail -20 $out/prof_bench.err; exit 1; }
tail -n 1 $out/prof_bench.jsonl | cut -c1-200
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --rehearse-one-gpu > $out/rehearse2.jsonl 2> $out/rehearse2.err || { tail -20 $out/rehearse2.err; exit 1; }
tail -n 1 $out/rehearse2.jsonl | cut -c1-300
