#!/bin/bash
# round 5 GPU pass 20: in-place SipHash transcript -- full GPU suite, sum-check bench, C4 quick bench
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu20
mkdir -p $out
timeout -k 10 1500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $out/pytest_gpu.txt 2>&1 || { tail -30 $out/pytest_gpu.txt; exit 1; }
tail -2 $out/pytest_gpu.txt
for rep in 1 2; do
  timeout -k 10 200 python3 -u tools/sc_bench.py 20,24 > $out/sc_$rep.json 2> $out/sc_$rep.err || { cat $out/sc_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/sc_$rep.json')); print({k: (v['ms'], v['kernel_ms']) for k, v in d.items()})"
  timeout -k 10 200 python3 -u bench.py --no-extras --steps 10 --warmup 3 > $out/c4_$rep.jsonl 2> $out/c4_$rep.err || exit 1
  python3 -c "import json; d=json.loads(open('$out/c4_$rep.jsonl').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['twist_last_prove_ms'])"
done
