#!/bin/bash
# round 4: field add/sub with carry builtins (TNS_FIELD_BI) and the 4-wave accumulation it allows
# -- C4 bench and C2 MSM, default library vs libtns_bi.so (3 waves) vs libtns_bi4.so (4 waves)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r04_fieldbi
mkdir -p $out
L=$GRAFT_REPO_ROOT/multilinear-map-cryptography_amd
for rep in 1 2; do
  for v in default bi bi4; do
    if [ $v = default ]; then lib=$L/libtns.so; else lib=$L/libtns_$v.so; fi
    TNS_LIB=$lib timeout -k 10 200 python3 -u bench.py --no-extras --steps 10 --warmup 3 > $out/c4_${v}_$rep.jsonl 2> $out/c4_${v}_$rep.err || exit $?
    TNS_LIB=$lib timeout -k 10 100 python3 tools/msm_trace.py 20 20 > $out/c2_${v}_$rep.txt 2>&1 || exit $?
    echo "$v rep $rep C4: $(python3 -c "import json; d=json.loads(open('$out/c4_${v}_$rep.jsonl').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['avg_launch_ms'], d['stages_ms_per_step']['msm_accumulate'])")  C2: $(tail -n 1 $out/c2_${v}_$rep.txt)"
  done
done
