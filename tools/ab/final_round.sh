#!/bin/bash
# End-of-round evidence on one GPU (round 6): GPU suite + smoke, the bench as the driver runs it,
# the rocprofv3 kernel-trace/stats pass of the C4 bench (roofline cross-check), FETCH_SIZE /
# WRITE_SIZE passes (pmc_traffic), the 2- and 4-rank sharded rehearsals.
#   tools/ab/final_round.sh <tag>
set -uo pipefail
tag=${1:-final}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/final_$tag
mkdir -p $out
timeout -k 10 1100 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $out/pytest_gpu.txt 2>&1 || { tail -30 $out/pytest_gpu.txt; exit 1; }
tail -1 $out/pytest_gpu.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || { tail -20 $out/smoke.txt; exit 1; }
tail -1 $out/smoke.txt
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $out/bench_driverargs.jsonl 2> $out/bench_driverargs.err || { tail -20 $out/bench_driverargs.err; exit 1; }
tail -c 300 $out/bench_driverargs.jsonl; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/ks -o run --output-format csv -- python3 bench.py --no-extras --steps 5 --warmup 2 > $out/bench_prof.jsonl 2> $out/bench_prof.err || { tail -20 $out/bench_prof.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o run --output-format csv -- python3 bench.py --no-extras --steps 2 --warmup 1 > $out/fetch.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $out/write -o run --output-format csv -- python3 bench.py --no-extras --steps 2 --warmup 1 > $out/write.log 2>&1 || exit 1
python3 tools/pmc_summary.py $out 5 > $out/pmc_traffic.json 2> $out/pmc_summary.err || { cat $out/pmc_summary.err; exit 1; }
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29551 bench.py --gpus 2 --steps 3 --warmup 1 --rehearse-one-gpu > $out/rehearse2.jsonl 2> $out/rehearse2.err || { tail -20 $out/rehearse2.err; exit 1; }
timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29552 bench.py --gpus 4 --steps 3 --warmup 1 --rehearse-one-gpu > $out/rehearse4.jsonl 2> $out/rehearse4.err || { tail -20 $out/rehearse4.err; exit 1; }
echo done
