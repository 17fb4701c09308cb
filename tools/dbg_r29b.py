"""Debug: the half_equal skewed MSM (tests/test_gpu_parity.py) with the radix-2^29 table
accumulation, repeated, against the per-window (radix-2^32) path and the trapdoor value."""
import os, sys
root = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, os.path.join(root, "multilinear-map-cryptography_amd"))
sys.path.insert(0, root)
import numpy as np
import twist_and_shout as ts
from oracle import pyoracle as po
R = po.R_MOD
pp, _ = ts.setup_params(18)
n = 1 << 20
rng = np.random.default_rng(1)
a = rng.integers(0, 2**63, size=(n // 2, 4), dtype=np.uint64) * 2 + rng.integers(0, 2, size=(n // 2, 4), dtype=np.uint64)
a[:, 3] &= np.uint64(0x0FFFFFFFFFFFFFFF)
pattern = sys.argv[1] if len(sys.argv) > 1 else "half_equal"
if pattern == "half_equal":
    vals = [R - 7] * (n // 2) + ts.from_mont(a)
elif pattern == "all_equal":
    vals = [R - 7] * n
else:
    vals = ts.from_mont(np.concatenate([a, a]))
c = ts.to_mont(vals)
outs = [ts.msm(pp.commitment_params, c) for _ in range(3)]
ctx = ts.Context.get(0)
ctx.set_msm_tables(False)
pw = ts.msm(pp.commitment_params, c)
ctx.set_msm_tables(True)
tau = pp.commitment_params.tau
s = 0
for v in reversed(vals):
    s = (s * tau + v) % R
want = po.affine_mul(po.G1_GEN, s)
print(pattern, "tables:", [str(o[0])[:12] for o in outs], "per-window:", str(pw[0])[:12], "want:", str(want[0])[:12], flush=True)
