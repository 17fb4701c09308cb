#!/bin/bash
# round 5 GPU pass 3: sum-check kernel v2 (tests, bench, trace, SQ counters), C2 state test, MSM plan
# A/B for the narrow trace commitments (forced c), sort tile variant
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu3
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sumcheck.py tests/test_gpu_parity.py -k "sumcheck" > $out/pytest_sc.txt 2>&1 || { tail -30 $out/pytest_sc.txt; exit 1; }
tail -2 $out/pytest_sc.txt
timeout -k 10 200 python3 -u tools/sc_bench.py 20,24 > $out/sc_bench.json 2> $out/sc_bench.err || { cat $out/sc_bench.err; exit 1; }
cat $out/sc_bench.json
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/sc_trace -o run --output-format csv -- python3 tools/sc_bench.py 20,24 > $out/sc_trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $out/sc_sq -o run --output-format csv -- python3 tools/sc_bench.py 24 > $out/sc_sq.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/c2_state.py > $out/c2_state.jsonl 2> $out/c2_state.err || { tail $out/c2_state.err; exit 1; }
cat $out/c2_state.jsonl
timeout -k 10 900 bash tools/ab/r05_ab_env.sh msmc 2 - TNS_MSM_C=16 TNS_MSM_C=12 TNS_MSM_C=14 || exit 1
timeout -k 10 600 bash tools/ab/r05_ab_libs.sh tiles 2 t16k || exit 1
