#!/bin/bash
# round 5 evidence pass 1: C2 kernel traces of the r03 tree and this tree (same box), the C4 step
# timeline, the SQ counter pass and FETCH/WRITE passes of one C4 step on this tree.
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_prof1
mkdir -p $out
for v in r03 head; do
  if [ $v = r03 ]; then d=ab/r03; else d=.; fi
  (cd $d && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/c2_$v -o run --output-format csv -- python3 tools/msm_trace.py 20 20) > $out/c2_$v.log 2>&1 || exit $?
  tail -n 1 $out/c2_$v.log
done
bash tools/c4_step_trace.sh r05_head || exit $?
cp -r gpurun_out/c4trace_r05_head $out/ 2>/dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $out/sq -o run --output-format csv -- python3 bench.py --no-extras --steps 1 --warmup 0 > $out/sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD -d $out/sq2 -o run --output-format csv -- python3 bench.py --no-extras --steps 1 --warmup 0 > $out/sq2.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $out/pmc_$c -o run --output-format csv -- python3 bench.py --no-extras --steps 1 --warmup 0 > $out/pmc_$c.log 2>&1 || exit $?
done
echo done
