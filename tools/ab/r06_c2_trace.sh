#!/bin/bash
# round 6: kernel timeline of the C2 MSM (2^20 Fr::rand scalars over setup_params(18)'s basis)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06_c2_trace
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace -d $out/tr -o run --output-format csv -- python3 tools/c2c3_bench.py > $out/run.txt 2> $out/run.err || { tail -20 $out/run.err; exit 1; }
cat $out/run.txt
