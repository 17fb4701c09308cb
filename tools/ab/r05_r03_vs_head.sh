#!/bin/bash
# round 5: same-box A/B of the round-3 final tree (c6ed2ce, built under ab/r03) against this tree,
# the driver's bench arguments, alternating:  tools/ab/r05_r03_vs_head.sh [reps]
set -uo pipefail
reps=${1:-3}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05_ab_r03_vs_head
mkdir -p $out
# what the box's sysfs offers for the device-state record
for f in /sys/class/drm/card*/device; do
  echo "== $f -> $(readlink -f $f)"
  for g in pp_dpm_sclk pp_dpm_mclk pp_dpm_fclk power_dpm_force_performance_level serial_number unique_id; do
    echo "-- $g: $(cat $f/$g 2>&1 | tr '\n' ' ' | cut -c1-200)"
  done
  for h in $f/hwmon/hwmon*; do
    for g in power1_cap power1_average power1_input temp1_input temp2_input temp3_input; do
      echo "-- $h/$g: $(cat $h/$g 2>&1)"
    done
  done
done > $out/sysfs_probe.txt 2>&1
# background sampler: every card's current sclk / power every 0.5 s over both trees' runs
( while true; do
    ts=$(date +%s.%N)
    for f in /sys/class/drm/card*/device; do
      s=$(grep '\*' $f/pp_dpm_sclk 2>/dev/null | tr -d '\n'); p=$(cat $f/hwmon/hwmon*/power1_average 2>/dev/null || cat $f/hwmon/hwmon*/power1_input 2>/dev/null)
      [ -n "$s$p" ] && echo "$ts $(basename $(readlink -f $f)) sclk[$s] power_uw[$p]"
    done
    sleep 0.5
  done ) > $out/sysfs_samples.txt 2>&1 &
sampler=$!
trap 'kill $sampler 2>/dev/null' EXIT
for rep in $(seq 1 $reps); do
  for v in r03 head; do
    if [ $v = r03 ]; then d=ab/r03; else d=.; fi
    echo "$(date +%s.%N) $v rep $rep start" >> $out/marks.txt
    (cd $d && timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5) > $out/${v}_$rep.jsonl 2> $out/${v}_$rep.err || exit $?
    echo "$(date +%s.%N) $v rep $rep done" >> $out/marks.txt
    echo "$v rep $rep: $(python3 -c "
import json; d=json.loads(open('$out/${v}_$rep.jsonl').read().strip().splitlines()[-1])
ds=d.get('device_state') or {}
print(d['ms_per_step'], d.get('ms_per_step_dropin'), d['roofline']['avg_launch_ms'], d['stages_ms_per_step'].get('msm_accumulate'),
      d['stages_ms_per_step'].get('msm_sort'), d.get('msm_ms_2^20'), (ds.get('during') or {}).get('sclk_mhz'), (ds.get('during') or {}).get('power_w'))")"
  done
done
