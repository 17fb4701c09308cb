import os, sys
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "multilinear-map-cryptography_amd"))
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import twist_and_shout as ts
logn = int(sys.argv[1]) if len(sys.argv) > 1 else 20
n = 1 << logn; L = logn - 2
pp, _ = ts.setup_params(L)
pp.commitment_params.srs.prepare_lagrange(n)
addr, val, isw = ts.bench_trace(1 << L, n)
ctx = pp.commitment_params.srs.ctx
d = [ts.DeviceBuffer(ctx, x) for x in (addr, val, isw)]
res = [ts.twist_proof_from_raw(ts.twist_prove_resident(pp, *d, n)) for _ in range(2)]
dro = [ts.Twist(pp).prove_soa(addr, val, isw) for _ in range(2)]
def show(tag, g):
    print(tag, hex(g.address_commitment.commitment[0])[:18], hex(g.value_commitment.commitment[0])[:18],
          hex(g.opening_proofs[0].proof[0])[:18], hex(g.opening_proofs[1].proof[0])[:18], flush=True)
for i, g in enumerate(res): show("res%d" % i, g)
for i, g in enumerate(dro): show("dro%d" % i, g)
