#!/bin/bash
# Round evidence in one GPU call: the default bench line (extras + CPU baseline), a
# rocprofv3 kernel-trace summary, and FETCH_SIZE / WRITE_SIZE passes (separate runs).
#   tools/round_profile.sh <tag>
set -euo pipefail
tag=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/prof_$tag
mkdir -p $out
timeout -k 10 400 python3 -u bench.py > $out/bench.jsonl 2> $out/bench.err
cat $out/bench.jsonl
args=("--no-extras" "--steps" "2" "--warmup" "1")
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/ks -o run --output-format csv -- python3 bench.py "${args[@]}" > $out/ks.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o run --output-format csv -- python3 bench.py "${args[@]}" > $out/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $out/write -o run --output-format csv -- python3 bench.py "${args[@]}" > $out/write.log 2>&1
echo profile-done
