#!/bin/bash
# the TNS_BS_BITS=last+1 parity variant (every pattern), and a kernel trace showing the 1024-bin kernels ran
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu27
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "sort_variants" > $out/pytest.txt 2>&1 || { tail -30 $out/pytest.txt; exit 1; }
tail -1 $out/pytest.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 -m pytest -x -q -m gpu tests/test_gpu_parity.py -k "sort_variants and last and full" > $out/prof.txt 2>&1 || { tail -30 $out/prof.txt; exit 1; }
tail -1 $out/prof.txt
find $out/prof -name '*kernel_stats.csv' | head -1 | xargs cut -d, -f1 | grep -E "k_bs_(count|scatter)" | head -20
