#!/bin/bash
# round 6: the persistent sum-check tail's solo rounds (block 0 alone below SC_SOLO_PAIRS pairs)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/ab/r06_ab_sc.sh 2 so0 so64 so256 so1k || exit 1
out=gpurun_out/r06_sc_tail_solo
mkdir -p $out
TNS_LIB=$GRAFT_REPO_ROOT/multilinear-map-cryptography_amd/libtns_sctr.so timeout -k 10 120 python3 tools/sc_trace.py 20 3 > $out/run.txt 2> $out/trace.txt || { tail $out/trace.txt; exit 1; }
cat $out/run.txt; tail -n 14 $out/trace.txt
