#!/bin/bash
# round-3: per-kernel stats of the C4 bench under each env setting in $AB (";"-separated, "-" =
# defaults), alternating twice; prints the sort kernels' average durations side by side
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${OUT:-r03sp}
mkdir -p $out
IFS=';' read -ra VARS <<< "${AB:--}"
for rep in 1 2; do
  for v in "${VARS[@]}"; do
    tag=$(echo "$v" | tr -c 'A-Za-z0-9_=\n' '_')_$rep
    ( [ "$v" != "-" ] && export $v; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$tag -o run --output-format csv -- python3 -u bench.py --no-extras --steps ${STEPS:-5} --warmup 2 > $out/$tag.jsonl 2> $out/$tag.err )
    rc=$?; [ $rc = 0 ] || { echo "prof $v rc=$rc"; tail -5 $out/$tag.err; exit $rc; }
    python3 - "$out/$tag" "$v" <<'PY'
import csv, glob, json, sys
d = sys.argv[1]
f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0]
b = json.loads(open(d + ".jsonl").read().strip().splitlines()[-1])
print("== %s: %.3f ms/step" % (sys.argv[2], b["ms_per_step"]))
tot = 0.0
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if "k_bs_" in n or "trampoline" in n or "k_accumulate" in n:
        print("  %-60s %5s %9.1f us avg %9.1f ms tot" % (n[:60], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
        if "k_accumulate" not in n:
            tot += float(r["TotalDurationNs"]) / 1e6
print("  sort kernels total %.2f ms" % tot)
PY
  done
done
