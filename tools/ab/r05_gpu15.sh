#!/bin/bash
# round 5 GPU pass 15: persistent sum-check tail with relaxed polls (tests; range x blocks A/B)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu15
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sumcheck.py tests/test_gpu_parity.py -k "sumcheck" > $out/pytest_sc.txt 2>&1 || { tail -30 $out/pytest_sc.txt; exit 1; }
tail -1 $out/pytest_sc.txt
for rep in 1 2; do
  for v in "13 256" "0 256" "11 256" "13 64" "13 1024" "15 256" "17 512"; do
    set -- $v
    TNS_SC_TAIL_LOG=$1 TNS_SC_TAIL_BLOCKS=$2 timeout -k 10 200 python3 -u tools/sc_bench.py 20,24 > $out/sc_$1_$2_$rep.json 2> $out/sc_$1_$2_$rep.err || { cat $out/sc_$1_$2_$rep.err; exit 1; }
    echo "tail<=2^$1 blocks<=$2 $rep $(python3 -c "import json; d=json.load(open('$out/sc_$1_$2_$rep.json')); print({k: (v['ms'], v['kernel_ms'], v['hbm_frac']) for k, v in d.items()})")"
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 tools/sc_bench.py 20,24 > $out/trace.log 2>&1 || exit 1
