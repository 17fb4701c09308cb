#!/bin/bash
# round 5 evidence pass 2 (final tree): the bench as the driver runs it, twice; rocprofv3 kernel stats
# of the same command (--no-extras); sum-check trace; one C4 step timeline
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_final2
mkdir -p $out
for rep in 1 2; do
  timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_$rep.jsonl 2> $out/bench_$rep.err || { tail -20 $out/bench_$rep.err; exit 1; }
  tail -n 1 $out/bench_$rep.jsonl | cut -c1-200
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-extras > $out/prof_bench.jsonl 2> $out/prof_bench.err || { tail -20 $out/prof_bench.err; exit 1; }
tail -n 1 $out/prof_bench.jsonl | cut -c1-200
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/sc_trace -o run --output-format csv -- python3 tools/sc_bench.py 20,24 > $out/sc_trace.log 2>&1 || exit 1
bash tools/c4_step_trace.sh r05_final2 || exit 1
