#!/bin/bash
# round 5: C4 bench (no extras) + C2 MSM, the default library vs variant builds (libtns_<tag>.so),
# alternating on one box:  tools/ab/r05_ab_libs.sh <name> <reps> <tag>...
set -uo pipefail
name=$1; reps=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_ab_$name
mkdir -p $out
L=$GRAFT_REPO_ROOT/multilinear-map-cryptography_amd
for rep in $(seq 1 $reps); do
  for v in default "$@"; do
    if [ $v = default ]; then lib=$L/libtns.so; else lib=$L/libtns_$v.so; fi
    TNS_LIB=$lib timeout -k 10 200 python3 -u bench.py --no-extras --steps 10 --warmup 3 > $out/c4_${v}_$rep.jsonl 2> $out/c4_${v}_$rep.err || exit $?
    TNS_LIB=$lib timeout -k 10 100 python3 tools/msm_trace.py 20 20 > $out/c2_${v}_$rep.txt 2>&1 || exit $?
    echo "$v rep $rep C4: $(python3 -c "import json; d=json.loads(open('$out/c4_${v}_$rep.jsonl').read().strip().splitlines()[-1]); s=d['stages_ms_per_step']; print(d['ms_per_step'], d['roofline']['avg_launch_ms'], s.get('msm_sort'), s.get('msm_accumulate'), (d['device_state']['valu_clock_after_steps'] or {}).get('median_mhz'))")  C2: $(tail -n 1 $out/c2_${v}_$rep.txt)"
  done
done
