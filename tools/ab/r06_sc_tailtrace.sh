#!/bin/bash
# round 6: the persistent sum-check tail's per-round timeline (TNS_SC_TRACE=1 build libtns_sctr.so)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06_sc_tail
mkdir -p $out
TNS_LIB=$GRAFT_REPO_ROOT/multilinear-map-cryptography_amd/libtns_sctr.so timeout -k 10 120 python3 tools/sc_trace.py 20 3 > $out/run.txt 2> $out/trace.txt || { tail $out/trace.txt; exit 1; }
cat $out/run.txt
tail -n 40 $out/trace.txt
