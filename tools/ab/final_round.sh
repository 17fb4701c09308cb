#!/bin/bash
# End-of-session evidence on one GPU: 2-rank sharded rehearsal, kernel-trace stats + HBM
# counters of the C4 bench, the C2 MSM's kernel timeline, and the bench as the driver runs it.
#   tools/ab/final_round.sh <tag>
set -euo pipefail
tag=${1:-final}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/rehearse2.sh $tag
bash tools/profile_round.sh $tag --stage-steps 0
python3 tools/pmc_summary.py gpurun_out/prof_$tag 3 > gpurun_out/pmc_traffic_$tag.json
bash tools/ab/msm_ks.sh c2$tag 20
python3 tools/trace_tail.py gpurun_out/msm_c2$tag/run_kernel_trace.csv k_scalar_bits > gpurun_out/msm_c2${tag}_tail.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_driver_$tag.jsonl 2> gpurun_out/bench_driver_$tag.err
tail -c 400 gpurun_out/bench_driver_$tag.jsonl
