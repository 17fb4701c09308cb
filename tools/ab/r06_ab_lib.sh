#!/bin/bash
# round 6: C4 (driver steps, no extras) with the default library vs build variants libtns_<tag>.so,
# alternating on one box:  tools/ab/r06_ab_lib.sh <name> <reps> <tag>...
set -uo pipefail
name=$1; reps=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06_ab_$name
mkdir -p $out
L=$GRAFT_REPO_ROOT/multilinear-map-cryptography_amd
for rep in $(seq 1 $reps); do
  for v in default "$@"; do
    if [ $v = default ]; then lib=$L/libtns.so; else lib=$L/libtns_$v.so; fi
    TNS_LIB=$lib timeout -k 10 200 python3 -u bench.py --no-extras --steps 20 --warmup 5 > $out/c4_${v}_$rep.jsonl 2> $out/c4_${v}_$rep.err || { tail -5 $out/c4_${v}_$rep.err; exit 1; }
    echo "$v rep $rep: $(python3 -c "
import json; d=json.loads(open('$out/c4_${v}_$rep.jsonl').read().strip().splitlines()[-1]); s=d['stages_ms_per_step']
print('step', d['ms_per_step'], 'commit', d['twist_last_prove_ms']['commit'], 'acc', d['roofline']['avg_launch_ms'], 'sort', s.get('msm_sort'), 'fixup', s.get('msm_fixup'), 'reduce', s.get('msm_reduce'), 'open_scan', s.get('open_scan'))")" | tee -a $out/summary.txt
  done
done
