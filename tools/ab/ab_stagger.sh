set -euo pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TNS_MSM_STAGGER=0 timeout -k 10 200 python -u bench.py --no-extras --steps 4 > gpurun_out/ab0.jsonl 2>gpurun_out/ab0.err
TNS_MSM_STAGGER=1 timeout -k 10 200 python -u bench.py --no-extras --steps 4 > gpurun_out/ab1.jsonl 2>gpurun_out/ab1.err
python3 -c "
import json
for f in ['ab0','ab1']:
    d=json.load(open('gpurun_out/%s.jsonl'%f)); print(f, d['ms_per_step'], d['twist_last_prove_ms'])"
