#!/bin/bash
# round-3 GPU pass: chain-fusion probe variants, the GPU parity suite, the default bench line
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r03g1
mkdir -p $out
for b in tools/chainfuse_dtns_mul_cios tools/chainfuse_dtns_no_field_asm tools/chainfuse_dtns_mul_ciosdtns_no_field_asm; do
  echo "== $b" >> $out/chainfuse.txt
  timeout -k 10 120 $b >> $out/chainfuse.txt 2>&1 || { echo "probe rc=$?"; exit 1; }
done
grep -v "^  [ci]\|^  pre\|^  inv" $out/chainfuse.txt
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?
tail -5 $out/pytest_gpu.log
[ $rc = 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > $out/bench.jsonl 2> $out/bench.err
echo "bench rc=$?"
tail -c 1500 $out/bench.jsonl
