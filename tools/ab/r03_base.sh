#!/bin/bash
# round-3 start: baseline bench (driver arguments), the chain-fusion probe, host CPU facts
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03base
mkdir -p $out
{ nproc; python -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; lscpu | grep -E "Model name|^CPU\(s\)|Thread|Socket"; free -g | head -2; } > $out/host.txt 2>&1
timeout -k 10 120 tools/chainfuse > $out/chainfuse.txt 2>&1 || { echo "chainfuse rc=$?"; cat $out/chainfuse.txt; exit 1; }
cat $out/chainfuse.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $out/bench.jsonl 2> $out/bench.err
echo "bench rc=$?"
tail -c 600 $out/bench.jsonl
