#!/bin/bash
# full GPU pass: parity suite, the default bench line (driver arguments), rocprofv3 kernel stats
set -uo pipefail
tag=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03_$tag
mkdir -p $out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?
tail -3 $out/pytest_gpu.log
[ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $out/bench.jsonl 2> $out/bench.err
rc=$?
echo "bench rc=$rc"
[ $rc = 0 ] || exit $rc
python3 -c "import json;d=json.loads(open('$out/bench.jsonl').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d.get('twist_ops_per_sec_dropin'),d.get('ms_per_step_coefficient_route'),d.get('msm_ms_2^20'),d.get('shout_ms_2^20'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/ks -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-extras > $out/ks.log 2>&1
echo "rocprof rc=$?"
find $out/ks -name "*kernel_stats*" | head -2
