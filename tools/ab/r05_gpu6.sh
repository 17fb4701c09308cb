#!/bin/bash
# round 5 GPU pass 6: sum-check round kernel code size (unrolled points vs point loop vs product calls):
# SQ / instruction-cache counters, then alternating timings; C2 over a 2^20- vs 2^22-point SRS traced
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu6
mkdir -p $out
L=$GRAFT_REPO_ROOT/multilinear-map-cryptography_amd
for v in nostage3 xloop3; do
  TNS_LIB=$L/libtns_$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQC_ICACHE_REQ SQC_ICACHE_MISSES -d $out/pmc1_$v -o run --output-format csv -- python3 tools/sc_bench.py 24 > $out/pmc1_$v.log 2>&1 || exit 1
  TNS_LIB=$L/libtns_$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQC_ICACHE_HITS SQ_IFETCH SQ_INSTS_VMEM_RD -d $out/pmc2_$v -o run --output-format csv -- python3 tools/sc_bench.py 24 > $out/pmc2_$v.log 2>&1 || exit 1
  echo "== $v"
  for p in pmc1 pmc2; do python3 tools/pmc_view.py $(ls $out/${p}_$v/*counter_collection.csv | head -1) k_sc_round_poly; done
done
for rep in 1 2 3; do
  for v in nostage3 xloop3 xloop4 xcall; do
    TNS_LIB=$L/libtns_$v.so timeout -k 10 200 python3 -u tools/sc_bench.py 20,24 > $out/sc_${v}_$rep.json 2> $out/sc_${v}_$rep.err || { cat $out/sc_${v}_$rep.err; exit 1; }
    echo "$v $rep $(python3 -c "import json; d=json.load(open('$out/sc_${v}_$rep.json')); print({k: (v['ms'], v['kernel_ms'], v['hbm_frac']) for k, v in d.items()})")"
  done
done
for s in 18 20; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/c2_srs$s -o run --output-format csv -- python3 tools/msm_trace.py 20 20 $s > $out/c2_srs$s.log 2>&1 || exit 1
  tail -n 1 $out/c2_srs$s.log
done
