#!/bin/bash
# round-3 final evidence on one MI355X: GPU suite, driver-style bench, rocprofv3 kernel stats,
# PMC FETCH_SIZE / WRITE_SIZE passes (separate runs, per MI355X_MICROARCH.md), the 4-rank C5
# rehearsal on one GPU and smoke()
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${OUT:-r03fin}
mkdir -p $out
step() { echo "== $1"; }
step pytest
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; tail -2 $out/pytest_gpu.log; [ $rc = 0 ] || exit $rc
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1
rc=$?; tail -1 $out/smoke.txt; [ $rc = 0 ] || exit $rc
step bench
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $out/bench.jsonl 2> $out/bench.err
rc=$?; [ $rc = 0 ] || { tail -5 $out/bench.err; exit $rc; }
head -c 400 $out/bench.jsonl; echo
step prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 -u bench.py --steps 20 --warmup 5 --no-extras > $out/bench_prof.jsonl 2> $out/bench_prof.err
rc=$?; [ $rc = 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  d=$out/pmc/$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
  mkdir -p $d
  step "pmc $c"
  timeout -s KILL 240 rocprofv3 --pmc $c -d $d -o run --output-format csv -- python3 bench.py --no-extras --steps 2 --warmup 0 --stage-steps 0 > $d/bench.log 2>&1
  rc=$?; [ $rc = 0 ] || { tail -5 $d/bench.log; exit $rc; }
done
step rehearse4
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29534 bench.py --gpus 4 --steps 2 --warmup 1 --rehearse-one-gpu > $out/rehearse4.jsonl 2> $out/rehearse4.err
rc=$?; [ $rc = 0 ] || { tail -5 $out/rehearse4.err; exit $rc; }
tail -1 $out/rehearse4.jsonl | cut -c1-500
echo done
