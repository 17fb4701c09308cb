#!/bin/bash
# round 5 GPU pass 13: mad + carry pair peak at a measured clock (macbench between two clock probes);
# opening sorts side by side vs one after the other (TNS_SORT_OVERLAP)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_gpu13
mkdir -p $out
probe() { timeout -k 10 60 python3 -c "
import sys; sys.path.insert(0, 'multilinear-map-cryptography_amd')
import twist_and_shout as ts
print('clock probe', ts.clock_probe(ts.Context.get(0), 200.0), flush=True)"; }
probe > $out/clock_before.txt 2>&1 || exit 1
timeout -k 10 120 tools/macbench > $out/macbench.txt 2>&1 || exit 1
probe > $out/clock_after.txt 2>&1 || exit 1
cat $out/clock_before.txt $out/macbench.txt $out/clock_after.txt
for rep in 1 2; do
  for v in 1 0; do
    TNS_SORT_OVERLAP=$v timeout -k 10 200 python3 -u bench.py --no-extras --steps 10 --warmup 3 > $out/c4_ov${v}_$rep.jsonl 2> $out/c4_ov${v}_$rep.err || exit 1
    echo "overlap=$v rep $rep $(python3 -c "import json; d=json.loads(open('$out/c4_ov${v}_$rep.jsonl').read().strip().splitlines()[-1]); s=d['stages_ms_per_step']; print(d['ms_per_step'], s.get('msm_sort'), s.get('msm_accumulate'), (d['device_state']['valu_clock_after_steps'] or {}).get('median_mhz'))")"
  done
done
