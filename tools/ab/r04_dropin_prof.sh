#!/bin/bash
# round 4: drop-in Twist::prove at C4 (host buffers, PCIe) -- kernel + memory-copy trace, merged timeline
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04_dropin
mkdir -p $out
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace -d $out/tr -o run --output-format csv -- python3 tools/dropin_trace.py 22 3 > $out/run.log 2>&1 || exit $?
python3 tools/dropin_timeline.py $out/tr 0.05 > $out/timeline.txt 2>&1
tail -n 3 $out/timeline.txt
