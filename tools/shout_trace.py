"""C3 Shout::prove (2^20 squares table, 2^20 lookups i % 2^20, setup_params(18)) repeated, for
kernel traces:  rocprofv3 --kernel-trace -d gpurun_out/sh -o run --output-format csv -- python3 tools/shout_trace.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "multilinear-map-cryptography_amd"))
import twist_and_shout as ts  # noqa: E402

pp, _ = ts.setup_params(18)
ctx = ts.Context.get(0)
pp.commitment_params.srs.prepare_lagrange(1 << 20)
T = 1 << 20
entries = ts.fr_from_u64_array(np.arange(T, dtype=np.uint64) ** 2)
idx = np.arange(T, dtype=np.uint64)
d_e, d_i = ts.DeviceBuffer(ctx, entries), ts.DeviceBuffer(ctx, idx)
ts.shout_prove_resident(pp, d_e, T, d_i, T)
t = time.perf_counter()
for _ in range(3):
    ts.shout_prove_resident(pp, d_e, T, d_i, T)
print(f"shout 2^20: {(time.perf_counter() - t) / 3 * 1e3:.3f} ms", flush=True)
