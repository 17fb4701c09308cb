#!/usr/bin/env python3
"""bench.py -- Twist prover ops/s (C4 / C5) + KZG MSM G1-scalar-pairs/s at 2^20 (C2) on MI355X.

A "step" is one Twist::prove (src/twist.rs:107-252) of the synthetic read/write trace of
ProtocolBenchmarks (src/benchmarks.rs:88-99) with the trace already resident in HBM.

Workloads (BASELINE.json configs):
  * N = 1 (default): C4 = setup_params(22), MemoryTrace::new(2^22), 2^24 operations.
  * N > 1 (default): C5 = ONE proof of the 2^26-operation trace, setup_params(24), sharded over
    the N ranks (one process per GPU, torchrun): every rank holds a 2^26/N-op slice of the trace,
    of the Lagrange basis and of the SRS; the ranks exchange per-MSM partial sums, barycentric
    partials and fold values by allgather.  Total work fixed at C5: "scaling": "strong".
  * --strong: C5 at every N, including N = 1 (the same-work baseline of the strong curve);
    --weak: 2^24 operations per GPU (one N * 2^24-op proof); --independent: one C4 proof per rank.
`value` = operations of the proof(s) / the max over ranks of the timed region (barrier +
synchronize on both sides).  `--gpus N` without WORLD_SIZE starts the N rank processes itself
(torch.distributed.run on 127.0.0.1) before any GPU call; under torchrun WORLD_SIZE must equal N.

Extra fields (rank 0, N = 1): the drop-in rate (Twist::prove on host buffers through the C ABI,
PCIe included, over the same steps), the coefficient route (interpolation + coefficient KZG: the
only route for an SRS without tau, src/utils.rs:107), C2 MSM pairs/s at 2^20 (setup_params(18),
Fr::rand scalars from ChaCha20Rng([7;32])), C3 Shout lookups/s (2^20-entry table, 2^20 lookups),
the per-stage device-time breakdown (every stage timed by HIP events on 2 untimed steps after the
timed region), the roofline of the dominant kernel (HIP events around its launches, on the lane
stream it runs on, inside the timed steps -- the only events there; algorithmic bytes from
SURVEY.md 8(d)), and two CPU baselines on a bounded sample (oracle/fastcpu.c with the GPU path's
algorithms on every host core the process may use, and the C oracle restating the reference
algorithms).
"""

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "multilinear-map-cryptography_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

METRIC = "Twist prover ops/sec + KZG MSM G1-scalar-pairs/sec at 2^20, 1/2/4/8 GPU"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# v_mad_u64_u32 throughput of independent streams, measured by tools/mulbench2.hip on MI355X
# (profiles/r01_mulbench2.txt): the integer-VALU ceiling of the MSM accumulation; and the
# throughput of the mad + carry pairs each 32x32 MAC of the product needs (tools/macbench.hip,
# 8 waves per SIMD, profiles/r02_macbench.txt).
MAC_PEAK_T = 28.61
MAC_PAIR_PEAK_T = 17.78
MAC_PAIR_PEAK_MHZ = 2338.0  # the VALU clock macbench's pair peak was measured at (profiles/r05_macbench_clock.txt)
# multiply-adds per lazy XYZZ mixed addition (bn254.hpp xyzz_madd_lazy): 6 products (64 + 64
# reduction), 2 squares (36 + 64), Y3 as two products under one reduction (64 + 64 + 64)
MACS_PER_MADD = 6 * 128 + 2 * 100 + 192


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--log-ops", type=int, default=None,
                    help="operations of one proof, 2^k (default: C4 = 24 at N = 1, C5 = 26 at N > 1)")
    mode = ap.add_mutually_exclusive_group()
    mode.add_argument("--strong", action="store_true", help="C5 (one 2^26-op proof) at every N, N = 1 included")
    mode.add_argument("--weak", action="store_true", help="2^24 operations per GPU: one N * 2^24-op proof")
    ap.add_argument("--no-extras", action="store_true", help="skip C2/C3 extras and the CPU baseline")
    ap.add_argument("--cpu-ref-logs", default="4-9",
                    help="reference-algorithm oracle: time one proof at each 2^k ops, k in this range (a-b); "
                         "the O(N^3) time is fitted by a power law and extrapolated to 2^24 (labelled)")
    ap.add_argument("--cpu-fast-log-ops", type=int, default=24,
                    help="fast CPU baseline: one proof of 2^k operations (setup_params(k - 2)); 24 = C4 itself")
    ap.add_argument("--sumcheck-logs", default="20,24",
                    help="generic sum-check extra: degree-3 composition of three 2^k tables, for each k "
                         "(empty: skip)")
    ap.add_argument("--tau-free-log", type=int, default=20,
                    help="tau-less SRS extra: Lagrange basis from g1_powers alone at 2^k nodes, timed and "
                         "checked, then Twist::prove at 2^k ops on it (0: skip)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="fast CPU baseline threads (0: every core the process's affinity allows)")
    ap.add_argument("--dropin-steps", type=int, default=None,
                    help="drop-in (host-buffer) proofs timed after the resident steps (default: --steps)")
    ap.add_argument("--coef-steps", type=int, default=2,
                    help="coefficient-route proofs timed at N = 1 (0: skip)")
    ap.add_argument("--commit-basis", choices=["lagrange", "coefficients"], default="lagrange",
                    help="prove via the setup's Lagrange-basis SRS (default) or via interpolation + "
                         "coefficient KZG (the reference's route); identical proofs")
    ap.add_argument("--independent", action="store_true",
                    help="N>1: one independent trace per rank instead of one trace sharded over the ranks")
    ap.add_argument("--comm", choices=["torch", "rccl"], default="torch",
                    help="sharded proof exchange: torch.distributed process group (nccl = RCCL) or the "
                         "library's own RCCL communicator")
    ap.add_argument("--exchange-timeout", type=float, default=300.0,
                    help="N > 1: deadline in seconds of one exchange step of the sharded proof; a step that "
                         "misses it ends the run with exit status 3 and names the rank and step")
    ap.add_argument("--stall-rank", type=int, default=-1,
                    help="testing aid (N > 1): this rank sleeps --stall-s seconds before its first timed proof, "
                         "so the others meet the exchange deadline (exit status 3)")
    ap.add_argument("--stall-s", type=float, default=0.0)
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="testing aid: every rank on device 0 with a gloo process group (one-GPU box)")
    ap.add_argument("--no-msm-tables", action="store_true",
                    help="per-window MSM buckets instead of the fixed-base window tables")
    ap.add_argument("--no-table-steps", type=int, default=3,
                    help="N = 1 extra: C4 proofs timed with the MSM window tables off (per-window buckets, no "
                         "precomputation beyond the Lagrange basis), proof checked equal (0: skip)")
    ap.add_argument("--c5-steps", type=int, default=2,
                    help="N = 1 extra: C5 (one 2^26-op proof, setup_params(24)) on this one GPU, timed over "
                         "this many steps -- the same-work denominator of the N > 1 strong-scaling lines (0: skip)")
    ap.add_argument("--stage-steps", type=int, default=2,
                    help="untimed steps after the timed region that time every stage (stages_ms_per_step); "
                         "the timed steps time only the roofline kernel (two HIP events per launch)")
    ap.add_argument("--profile-all-timed", action="store_true",
                    help="A/B: time every stage inside the timed steps (the pre-round-2 behaviour)")
    return ap.parse_args()


def launch_ranks(args) -> int:
    """--gpus N without WORLD_SIZE: start the N rank processes (torch.distributed.run, one process
    per GPU, rendezvous on 127.0.0.1) as children -- before this process touches the GPU -- and
    return their exit code."""
    import socket
    import subprocess

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.rehearse_one_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    pg = None
    if world > 1:
        import torch
        import torch.distributed as dist

        if torch.cuda.is_available() and not args.rehearse_one_gpu:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", rank=rank, world_size=world)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        pg = dist
    return world, rank, local, pg


def barrier_sync(pg, local):
    if pg is not None:
        import torch

        if torch.cuda.is_available():
            torch.cuda.synchronize(local)
        pg.barrier()


def max_over_ranks(pg, local, x):
    if pg is None:
        return x
    import torch

    on_gpu = torch.cuda.is_available() and pg.get_backend() == "nccl"
    dev = torch.device("cuda", local) if on_gpu else torch.device("cpu")
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    pg.all_reduce(t, op=pg.ReduceOp.MAX)
    return float(t.item())


ROOF_KERNEL = "msm_accumulate"  # the dominant stage by device time (every stage timed: stages_ms_per_step)


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _dpm_current(text):
    """Current level of a pp_dpm_* table ('1: 2100Mhz *') as MHz."""
    if not text:
        return None
    for line in text.splitlines():
        if line.rstrip().endswith("*"):
            tok = line.split(":", 1)[-1].strip().rstrip("*").strip().lower().replace("mhz", "")
            try:
                return float(tok)
            except ValueError:
                return None
    return None


class DeviceState:
    """The card's clocks, power and temperature around the timed region (the driver's numbers
    differ box to box by several per cent; this is what tells a slow box from a slow build).
    Sources: hipDeviceProp_t (tns_device_info_get: rated clocks, PCI bus id) and the amdgpu sysfs
    files of that PCI device (pp_dpm_sclk / pp_dpm_mclk current levels, hwmon power cap, power,
    temperatures, the board serial as the box identifier); a sampler thread reads the current
    sclk / power / edge temperature every 100 ms while the steps run.  Missing files are null."""

    def __init__(self, ts, device):
        self.info = None
        try:
            self.info = ts.device_info(device)
        except Exception as e:  # the record is diagnostic; never fail the bench over it
            self.info = {"error": str(e)}
        bus = (self.info or {}).get("pci_bus_id")
        self.dev = f"/sys/bus/pci/devices/{bus}" if bus else None
        self.hwmon = None
        if self.dev and os.path.isdir(os.path.join(self.dev, "hwmon")):
            hw = sorted(os.listdir(os.path.join(self.dev, "hwmon")))
            if hw:
                self.hwmon = os.path.join(self.dev, "hwmon", hw[0])
        self.samples = []
        self._stop = None
        self._thread = None

    def _hw(self, name, scale):
        if not self.hwmon:
            return None
        v = _read(os.path.join(self.hwmon, name))
        try:
            return round(int(v) / scale, 2) if v is not None else None
        except ValueError:
            return None

    def snapshot(self):
        d = self.dev
        return {"t": round(time.time(), 3),
                "sclk_mhz": _dpm_current(_read(os.path.join(d, "pp_dpm_sclk"))) if d else None,
                "mclk_mhz": _dpm_current(_read(os.path.join(d, "pp_dpm_mclk"))) if d else None,
                "fclk_mhz": _dpm_current(_read(os.path.join(d, "pp_dpm_fclk"))) if d else None,
                "power_w": self._hw("power1_average", 1e6) or self._hw("power1_input", 1e6),
                "power_cap_w": self._hw("power1_cap", 1e6),
                "temp_edge_c": self._hw("temp1_input", 1e3),
                "temp_hotspot_c": self._hw("temp2_input", 1e3),
                "temp_mem_c": self._hw("temp3_input", 1e3),
                "perf_level": _read(os.path.join(d, "power_dpm_force_performance_level")) if d else None}

    def start(self):
        import threading

        self.begin = self.snapshot()
        self._stop = threading.Event()

        def run():
            while not self._stop.wait(0.1):
                s = self.snapshot()
                self.samples.append((s["sclk_mhz"], s["power_w"], s["temp_edge_c"]))

        self._thread = threading.Thread(target=run, daemon=True)
        self._thread.start()

    def stop(self):
        if self._thread is not None:
            self._stop.set()
            self._thread.join()
        self.end = self.snapshot()

    def record(self):
        def stat(i):
            xs = [s[i] for s in self.samples if s[i] is not None]
            if not xs:
                return None
            return {"min": min(xs), "mean": round(sum(xs) / len(xs), 1), "max": max(xs), "n": len(xs)}

        return {"device": self.info, "sysfs": self.dev if self.dev and os.path.isdir(self.dev) else None,
                "host": platform.node(), "board_serial": _read(os.path.join(self.dev, "serial_number")) if self.dev
                else None, "unique_id": _read(os.path.join(self.dev, "unique_id")) if self.dev else None,
                "start": getattr(self, "begin", None), "end": getattr(self, "end", None),
                "valu_clock_after_steps": getattr(self, "valu_clock", None),
                "during": {"sclk_mhz": stat(0), "power_w": stat(1), "temp_edge_c": stat(2),
                           "sampler": "every 100 ms over the timed region"}}


def read_stages(ts, ctx):
    stages = {}
    for s in ts.PROFILE_STAGES:
        ms, n, b = ts.profile_read(ctx, s)
        if n:
            stages[s] = {"ms": ms, "launches": n, "alg_bytes": b}
    return stages


def roofline_from_profile(ts, ctx):
    stages = read_stages(ts, ctx)
    if not stages:
        return None, stages
    dom = max(stages, key=lambda k: stages[k]["ms"])
    d = stages[dom]
    avg_s = d["ms"] / d["launches"] / 1e3
    per_launch = d["alg_bytes"] / d["launches"]
    achieved = per_launch / avg_s / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        try:
            with open(pmc) as f:
                traffic = json.load(f).get(dom, {}).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    roof = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 5), "traffic": traffic,
            "alg_bytes_per_launch": per_launch, "avg_launch_ms": round(avg_s * 1e3, 4),
            "note": "dominant stage by device time: k_accumulate, averaged over a step's 4 launches (2 "
                    "narrow-scalar commitments, 2 full-width openings); integer-VALU-bound (256-bit "
                    "Montgomery), so the HBM fraction is low by construction (compute position: the "
                    "'compute' object); the two MSMs of a commit/open pair accumulate one after the "
                    "other, so each launch's HIP-event duration is its own kernel time -- see DESIGN.md"}
    ex = ts.profile_read_ex(ctx, "msm_accumulate")
    if ex["ops"] and ex["busy_ms"]:
        tmacs = ex["ops"] * MACS_PER_MADD / (ex["busy_ms"] / 1e3) / 1e12
        roof["compute"] = {"kernel": "msm_accumulate", "bound": "valu (v_mad_u64_u32)", "unit": "T MAC/s",
                           "achieved": round(tmacs, 3), "peak": MAC_PEAK_T, "frac": round(tmacs / MAC_PEAK_T, 4),
                           "mac_carry_pair_peak": MAC_PAIR_PEAK_T,
                           "frac_of_pair_peak": round(tmacs / MAC_PAIR_PEAK_T, 4),
                           "madds": ex["ops"], "busy_ms": round(ex["busy_ms"], 3),
                           "note": f"mixed additions x {MACS_PER_MADD} MACs over the union of the stage's launch "
                                   "intervals; peak = measured independent v_mad_u64_u32 streams (tools/mulbench2.hip); "
                                   "each MAC of the 32-bit-limb product also needs a carry instruction, and mad + carry "
                                   "pairs peak at mac_carry_pair_peak (tools/macbench.hip, 8 waves/SIMD)"}
    return roof, stages


def cpu_reference_algorithms(logs):
    """The C oracle restating the reference algorithms (O(N^3) Lagrange interpolation, per-term
    commit, closure sum-check; single-threaded as the reference's .iter()) timed on one proof of
    the ProtocolBenchmarks trace at each 2^k ops (setup_params(k), MemoryTrace::new(2^k)), a power
    law t = a N^b fitted to the three largest sizes and extrapolated -- labelled as such -- to
    C4's 2^24 operations (baseline (1))."""
    from oracle import coracle as co
    from oracle import pyoracle as po

    pts = []
    for k in logs:
        n_ops = 1 << k
        cp = co.setup_params(k)
        ops = po.benchmark_trace(n_ops, n_ops)
        t0 = time.perf_counter()
        st, _ = co.twist_prove(cp, ops)
        dt = time.perf_counter() - t0
        assert st == 0
        pts.append((k, dt))
    fit = pts[-3:] if len(pts) >= 3 else pts
    xs = np.array([k * np.log(2.0) for k, _ in fit])
    ys = np.log(np.array([t for _, t in fit]))
    b, a = np.polyfit(xs, ys, 1) if len(fit) > 1 else (3.0, ys[0] - 3.0 * xs[0])
    t24 = float(np.exp(a + b * 24 * np.log(2.0)))
    k_last, t_last = pts[-1]
    return {"value": round((1 << k_last) / t_last, 3), "unit": "ops/s", "cores": 1, "kind": "port",
            "sample": f"Twist::prove of the 2^{k_last}-op ProtocolBenchmarks trace (setup_params({k_last})) by the "
                      f"single-threaded C oracle restating the reference algorithms (O(N^3) interpolation); "
                      f"{t_last:.2f} s",
            "measured": [{"log_ops": k, "s": round(t, 4), "ops_per_sec": round((1 << k) / t, 3)} for k, t in pts],
            "fit": {"exponent": round(float(b), 3), "points": [k for k, _ in fit], "law": "t = a * N^b"},
            "extrapolated_2^24": {"s": round(t24, 1), "days": round(t24 / 86400, 1),
                                  "ops_per_sec": float(f"{(1 << 24) / t24:.4g}"),
                                  "note": "EXTRAPOLATED from the fit, not measured"}}


def host_cores():
    """(threads to use, note): every CPU the process's affinity allows, capped by the cgroup CPU
    quota when one is set (the GPU box grants 16 CPUs of time to a 1-GPU job on a 256-CPU host)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    n = min(aff, quota) if quota else aff
    return n, f"affinity {aff} CPUs, cgroup quota {quota if quota else 'none'} CPUs"


def cpu_baseline(ts, ctx, log_ops, threads=0, gpu_check=True, pp=None):
    """Fast CPU baseline (SURVEY 8(d) 'fast-CPU'): oracle/fastcpu.c proves Twist with the GPU
    path's algorithms (Lagrange-basis KZG, Pippenger MSM, fold sum-check) on every host core the
    process may use.  Bounded sample: one 2^log_ops-op proof of the src/benchmarks.rs:88-99 trace
    over setup_params(log_ops - 2); the basis [L_j(tau)]G is the device-built setup artefact
    (downloaded, not timed).  The proof is checked against the GPU's proof of the same trace."""
    from oracle import coracle as co

    n = 1 << log_ops
    L = log_ops - 2
    if pp is None or pp.log_size != L:
        pp, _ = ts.setup_params(L, device=ctx.device)
    pp.commitment_params.srs.prepare_lagrange(n)
    addr, val, isw = ts.bench_trace(1 << L, n)
    lag = pp.commitment_params.srs.lagrange_points(n)
    w = co.bary_weights(n)
    T, note = host_cores()
    if threads > 0:
        T = threads
    t0 = time.perf_counter()
    st, proof = co.fast_twist_prove(lag, w, pp.max_operations, addr, val, isw, T)
    dt = time.perf_counter() - t0
    assert st == 0
    out = {"value": round(n / dt, 1), "unit": "ops/s", "cores": T, "kind": "port",
           "sample": f"Twist::prove of a 2^{log_ops}-op trace (src/benchmarks.rs:88-99, setup_params({L})) with the "
                     f"GPU path's algorithms in C (oracle/fastcpu.c: Lagrange-basis KZG, Pippenger MSM, fold "
                     f"sum-check) on {T} host threads ({note}); {dt:.2f} s",
           "host_cpu": platform.processor() or platform.machine(), "host_nproc": os.cpu_count()}
    if gpu_check:
        g = ts.Twist(pp).prove_soa(addr, val, isw)
        same = (g.address_commitment.commitment == proof["address_commitment"]
                and g.value_commitment.commitment == proof["value_commitment"]
                and [q.proof for q in g.opening_proofs] == proof["opening_proofs"]
                and g.opening_point == proof["opening_point"])
        out["proof_identical_to_gpu"] = bool(same)
    return out


def sumcheck_generic(ts, ctx, logs):
    """SumCheck::prove (src/sumcheck.rs:56-110) of a non-zero degree-3 composition -- the Twist MLE
    shapes A V - O O V + 2 O over three random 2^k-entry tables resident in HBM -- timed end to
    end (k rounds: fused fold + round sums on the device, transcript on the host), with the round
    kernels' HIP-event time and algorithmic bytes (48 B per input entry and table once folded,
    32 B in round 0) giving their achieved GB/s against the 8 TB/s HBM peak."""
    R = ts.R_MOD
    terms = [(1, [0, 1]), (R - 1, [2, 2, 1]), (2, [2])]
    out = {}
    rng = np.random.default_rng(9)
    for k in logs:
        n = 1 << k
        tabs = []
        for _ in range(3):
            t = rng.integers(0, 2**63, size=(n, 4), dtype=np.uint64) * np.uint64(2)
            t[:, 3] &= np.uint64((1 << 60) - 1)
            tabs.append(ts.DeviceBuffer(ctx, t))
            del t
        claim = ts.SumCheck.composition_sum_resident(k, tabs, terms)
        sc = ts.SumCheck(k, claim)
        sc.prove_resident(tabs, terms, ts.Transcript(bytes(32)), raw=True)  # warm-up
        reps = 5
        # end to end with no profiling (HIP events around every round kernel cost ~10 us a round),
        # 20 proofs (mean and median per proof), then the round kernels' own time on separate proofs
        per = []
        for _ in range(20):
            t0 = time.perf_counter()
            sc.prove_resident(tabs, terms, ts.Transcript(bytes(32)), raw=True)
            per.append(time.perf_counter() - t0)
        dt = sum(per) / len(per)
        dt_med = float(np.median(per))
        ts.profile_enable(ctx, True)
        ts.profile_only(ctx, "sumcheck_round")
        for _ in range(reps):
            sc.prove_resident(tabs, terms, ts.Transcript(bytes(32)), raw=True)
        ex = ts.profile_read_ex(ctx, "sumcheck_round")
        ts.profile_only(ctx, None)
        ts.profile_enable(ctx, False)
        kms = ex["ms"] / reps
        gbs = ex["bytes"] / reps / (kms / 1e3) / 1e9 if kms else None
        # every round's algorithmic bytes (round 0 reads 64 B per pair and table, later rounds 192 B)
        # over the whole proof's wall time: the persistent tail's rounds carry no HIP events
        all_bytes = sum((64.0 if rr == 0 else 192.0) * (n >> (rr + 1)) * 3 for rr in range(k))
        out[f"2^{k}"] = {"ms": round(dt * 1e3, 3), "ms_median": round(dt_med * 1e3, 3), "proofs_timed": len(per),
                         "tables": 3, "degree": 3, "rounds": k,
                         "entries_per_sec": round(3 * n / dt, 1),
                         "kernel_ms": round(kms, 3), "kernel_launches": ex["launches"] // reps,
                         "alg_bytes": ex["bytes"] / reps,
                         "achieved_GBps": round(gbs, 1) if gbs else None,
                         "hbm_frac": round(gbs / HBM_PEAK_GBPS, 4) if gbs else None,
                         "end_to_end_GBps": round(all_bytes / dt / 1e9, 1),
                         "end_to_end_hbm_frac": round(all_bytes / dt / 1e9 / HBM_PEAK_GBPS, 4),
                         "kernel_note": "kernel_ms / alg_bytes / hbm_frac: the round kernels with HIP events (rounds "
                                        "before the persistent tail k_sc_tail, which spans the host's turns); "
                                        "end_to_end_*: every round's bytes over the proof's wall time",
                         "bound": "Fr multiply (3 products per composition point x 3 points -- g(1) comes from the claim -- + 2 per table per fold)"}
        del tabs
    return out


def tau_free_route(ts, ctx, log_n=20, steps=5):
    """The route an SRS WITHOUT tau ships with (src/utils.rs:61, :107 mark tau test-only): the
    one-time Lagrange basis from g1_powers alone (tns_srs_prepare_lagrange_from_powers, tfree.hip),
    timed at 2^log_n nodes and checked equal to the tau-derived basis, then Twist::prove of a
    2^log_n-op trace (src/benchmarks.rs:88-99, setup_params(log_n - 2)) on that tau-less SRS, timed
    beside the same proof on the setup SRS (identical proofs required).  The C4 basis (2^24) is the
    same build at 16x the nodes (145 s measured): once built it is bit-identical to
    the tau basis, so C4 proves at the headline rate on it."""
    import dataclasses

    n = 1 << log_n
    pp, _ = ts.setup_params(log_n - 2, device=ctx.device)
    srs = pp.commitment_params.srs
    srs.prepare_lagrange(n)
    want = srs.lagrange_points(n)
    cp = ts.CommitmentParams.from_g1_limbs(srs.download(len(srs)), device=ctx.device)  # g1_powers only
    t0 = time.perf_counter()
    cp.srs.prepare_lagrange_from_powers(n)
    t_basis = time.perf_counter() - t0
    same_basis = bool(np.array_equal(cp.srs.lagrange_points(n), want))
    del want
    pp_free = dataclasses.replace(pp, commitment_params=cp, _raw=None)
    addr, val, isw = ts.bench_trace(1 << (log_n - 2), n)
    d_addr, d_val, d_isw = ts.DeviceBuffer(ctx, addr), ts.DeviceBuffer(ctx, val), ts.DeviceBuffer(ctx, isw)
    proofs = {}

    def run(p, key):
        proofs[key] = ts.twist_prove_resident(p, d_addr, d_val, d_isw, n)

    t_tau = timed_proofs(lambda: run(pp, "tau"), steps, 1)
    t_free = timed_proofs(lambda: run(pp_free, "free"), steps, 1)
    same_proof = bytes(proofs["tau"]) == bytes(proofs["free"])
    return {"tau_free_basis_s_2^%d" % log_n: round(t_basis, 3),
            "tau_free_basis_equals_tau_basis": same_basis,
            "tau_free_twist_ops_per_sec_2^%d" % log_n: round(n / t_free, 1),
            "tau_free_twist_ms_2^%d" % log_n: round(t_free * 1e3, 3),
            "tau_twist_ms_2^%d" % log_n: round(t_tau * 1e3, 3),
            "tau_free_proof_identical": bool(same_proof),
            "tau_free_note": "SRS uploaded without tau (g1_powers only); Lagrange basis built from the powers "
                             "(transposed remainder tree, GLV twiddles) then Twist::prove at 2^%d ops on it; "
                             "C4's 2^24 basis is the same one-time build (145 s, DESIGN.md 2.8)" % log_n}


def sharded_msm(ts, ctx, comm, pg, local, rank, world, reps=10):
    """C2 at N ranks: KZGCommitment::commit of 2^20 Fr::rand scalars (ChaCha20Rng([7;32]),
    setup_params(18)) sharded over the ranks (tns_msm_sharded: per-rank partial MSM over its SRS
    share, allgather of the 96-byte partials); pairs/s = 2^20 / max over ranks of the time."""
    n = 1 << 20
    pp18, _ = ts.setup_params_shard(18, rank, world, ctx=ctx)
    first, cnt = ts.shard_slice(n, rank, world)
    sc = ts.fr_rand_batch(bytes([7] * 32), n)[first:first + cnt]
    d = ts.DeviceBuffer(ctx, np.ascontiguousarray(sc))
    for _ in range(2):
        ts.msm_sharded_resident(pp18.commitment_params, comm, d, cnt, n)
    barrier_sync(pg, local)
    t0 = time.perf_counter()
    for _ in range(reps):
        ts.msm_sharded_resident(pp18.commitment_params, comm, d, cnt, n)
    barrier_sync(pg, local)
    dt = max_over_ranks(pg, local, (time.perf_counter() - t0) / reps)
    return {"msm_pairs_per_sec_2^20": round(n / dt, 1), "msm_ms_2^20": round(dt * 1e3, 3),
            "msm_2^20_layout": f"2^20 pairs over {world} ranks, {cnt} per rank (tns_msm_sharded)"}


class exchange_guard:
    """A sharded step whose exchange fails (a peer rank stalled past the deadline, or the
    transport broke) ends the run: one JSON line on stderr naming this rank, the step and the
    communicator's diagnosis, then exit status 3 without waiting on the broken process group."""

    def __init__(self, ts, rank, what):
        self.ts, self.rank, self.what = ts, rank, what

    def __enter__(self):
        return self

    def __exit__(self, et, e, tb):
        if e is not None and isinstance(e, self.ts.DeviceError):
            kind = "deadline" if isinstance(e, self.ts.ExchangeTimeout) else "transport"
            print(json.dumps({"error": f"exchange {kind}", "rank": self.rank, "during": self.what,
                              "detail": str(e)}), file=sys.stderr, flush=True)
            os._exit(3)
        return False


def per_rank_exchange_record(pg, rank, dt, steps, s0, s1):
    """Every rank's timed-region ms per step and its exchange steps' host latency over the timed
    steps (tns_comm_stats deltas), gathered to every rank in rank order."""
    n = s1["exchanges"] - s0["exchanges"]
    tot = s1["total_s"] - s0["total_s"]
    by = s1["bytes_total"] - s0["bytes_total"]
    mine = {"rank": rank, "ms_per_step": round(dt / max(1, steps) * 1e3, 3),
            "exchanges_per_step": round(n / max(1, steps), 2),
            "mean_exchange_us": round(tot / n * 1e6, 1) if n else None,
            "max_exchange_us_so_far": round(s1["max_us"], 1) if s1["max_us"] is not None else None,
            "mean_exchange_bytes_per_rank": round(by / n, 1) if n else None,
            "max_exchange_bytes_per_rank": s1["max_bytes"]}
    if pg is None:
        return [mine]
    allv = [None] * pg.get_world_size()
    pg.all_gather_object(allv, mine)
    return allv


def c5_one_gpu(ts, ctx, local, steps):
    """C5's work on this one GPU: ONE Twist::prove of the 2^26-op trace over setup_params(24), trace
    resident -- the same-work N = 1 point of the strong-scaling curve the N > 1 lines (C5 sharded)
    are divided by.  Setup (SRS, Lagrange basis, window table) outside the timing, as for C4."""
    t0 = time.perf_counter()
    pp5, _ = ts.setup_params(24, device=local)
    pp5.commitment_params.srs.prepare_lagrange(1 << 26)
    n5 = 1 << 26
    addr, val, isw = ts.bench_trace(1 << 24, n5)
    d = [ts.DeviceBuffer(ctx, x) for x in (addr, val, isw)]
    del addr, val, isw
    setup_s = time.perf_counter() - t0
    t = timed_proofs(lambda: ts.twist_prove_resident(pp5, *d, n5), steps, 1)
    rec = {"workload": "C5 on one GPU: Twist::prove, 2^26-op trace, setup_params(24), trace resident",
           "steps": steps, "ms_per_step": round(t * 1e3, 3), "ops_per_sec": round(n5 / t, 2),
           "setup_s": round(setup_s, 2)}
    del d, pp5
    return rec


def timed_proofs(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    return (time.perf_counter() - t0) / max(1, steps)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world, rank, local, pg = dist_setup(args)
    import twist_and_shout as ts

    # (several processes on one GPU: no least-priority queue to starve behind the others')
    ctx = ts.Context.get(local, stream_priorities=not args.rehearse_one_gpu)
    sharded = world > 1 and not args.independent
    comm_cfg = None
    # operations of ONE proof: C4 (2^24) at N = 1, C5 (2^26, setup_params(24)) at N > 1
    if args.log_ops is not None:
        log_total = args.log_ops + (world.bit_length() - 1 if args.weak and sharded else 0)
    elif args.weak:
        log_total = 24 + (world.bit_length() - 1 if sharded else 0)
    elif args.strong or sharded:
        log_total = 26
    else:
        log_total = 24
    n_total = 1 << log_total
    n_ops = n_total // world if sharded else n_total  # per GPU
    L = log_total - 2  # setup_params(L): max_operations = 2^(L+2); memory size 2^L
    ctx.set_commit_basis(args.commit_basis == "lagrange")
    ctx.set_msm_tables(not args.no_msm_tables)
    t_setup = time.perf_counter()
    if sharded:  # one trace over all ranks: SRS share + basis slice per rank
        pp, _ = ts.setup_params_shard(L, rank, world, ctx=ctx)
    else:
        pp, _ = ts.setup_params(L, device=local)
    t_setup = time.perf_counter() - t_setup
    t_lag = time.perf_counter()
    if args.commit_basis == "lagrange":  # setup-time product, like g1_powers (not proving work)
        if sharded:
            pp.commitment_params.srs.prepare_lagrange_shard(n_total, rank, world)
        else:
            pp.commitment_params.srs.prepare_lagrange(n_ops)
    t_lag = time.perf_counter() - t_lag
    if sharded:
        first, count = ts.shard_slice(n_total, rank, world)
        addr, val, isw = ts.bench_trace_slice(1 << L, n_total, first, count)
        if args.comm == "rccl":
            uid = [ts.Comm.unique_id() if rank == 0 else None]
            pg.broadcast_object_list(uid, src=0)
            comm = ts.Comm.rccl(ctx, rank, world, uid[0], timeout_s=args.exchange_timeout)
        else:
            import torch

            on_gpu = torch.cuda.is_available() and not args.rehearse_one_gpu
            comm = ts.Comm.torch(device=torch.device("cuda", local) if on_gpu else None,
                                 timeout_s=args.exchange_timeout)
        # the rank count each transport itself reports must be --gpus (RCCL: ncclCommCount)
        info = comm.info()
        comm_cfg = {"kind": args.comm if args.comm == "rccl" else f"torch.distributed ({pg.get_backend()}) "
                                                                   "via the host-callback communicator",
                    "world_size_seen": info["seen_size"], "process_group_world_size": pg.get_world_size(),
                    "rank": info["rank"]}
        if info["seen_size"] != args.gpus or pg.get_world_size() != args.gpus or info["size"] != args.gpus:
            sys.exit(f"bench.py: the communicator sees {info['seen_size']} ranks (process group "
                     f"{pg.get_world_size()}) but --gpus {args.gpus}")
    else:
        count = n_ops
        addr, val, isw = ts.bench_trace(1 << L, n_ops)
    d_addr, d_val, d_isw = ts.DeviceBuffer(ctx, addr), ts.DeviceBuffer(ctx, val), ts.DeviceBuffer(ctx, isw)

    def prove():
        if sharded:
            with exchange_guard(ts, rank, "Twist::prove (sharded)"):
                return ts.twist_prove_sharded_resident(pp, comm, d_addr, d_val, d_isw, count, n_total)
        return ts.twist_prove_resident(pp, d_addr, d_val, d_isw, n_ops)

    for _ in range(args.warmup):
        prove()
    barrier_sync(pg, local)
    dstate = DeviceState(ts, local)
    ts.profile_enable(ctx, True)
    ts.profile_only(ctx, None if args.profile_all_timed else ROOF_KERNEL)
    cs0 = comm.stats() if sharded else None
    dstate.start()
    t0 = time.perf_counter()
    for step in range(args.steps):
        if sharded and step == 0 and rank == args.stall_rank and args.stall_s > 0:
            time.sleep(args.stall_s)  # (--stall-rank: rehearse the exchange deadline)
        prove()
    barrier_sync(pg, local)
    dt = time.perf_counter() - t0
    dstate.stop()
    try:  # the clock the card holds under the accumulation's kind of load, right after the steps
        dstate.valu_clock = ts.clock_probe(ctx, 60.0)
    except Exception as e:  # diagnostic only
        dstate.valu_clock = {"error": str(e)}
    if sharded:
        comm_cfg["per_rank"] = per_rank_exchange_record(pg, rank, dt, args.steps, cs0, comm.stats())
        comm_cfg["exchange_timeout_s"] = args.exchange_timeout
    breakdown = ctx.timing()
    roof, stages = roofline_from_profile(ts, ctx)
    clk = dstate.valu_clock.get("median_mhz") if isinstance(dstate.valu_clock, dict) else None
    if roof is not None and "compute" in roof and clk:
        # the pair peak scales with the VALU clock (DVFS under the power cap moves it box to box by
        # several %): the fraction at the clock this box held right after the timed steps
        cp = roof["compute"]
        peak_here = MAC_PAIR_PEAK_T * clk / MAC_PAIR_PEAK_MHZ
        cp["valu_clock_mhz"] = clk
        cp["mac_carry_pair_peak_at_clock"] = round(peak_here, 3)
        cp["frac_of_pair_peak_at_clock"] = round(cp["achieved"] / peak_here, 4)
    stage_steps = args.steps
    if not args.profile_all_timed and args.stage_steps > 0:  # every stage, on untimed steps
        ts.profile_enable(ctx, True)
        ts.profile_only(ctx, None)
        for _ in range(args.stage_steps):
            prove()
        barrier_sync(pg, local)
        stages = read_stages(ts, ctx)
        stage_steps = args.stage_steps
    ts.profile_only(ctx, None)
    ts.profile_enable(ctx, False)
    dt_max = max_over_ranks(pg, local, dt)
    total_ops = (n_total if sharded else world * n_ops) * args.steps
    value = total_ops / dt_max
    if sharded:
        workload = (f"{'C5' if log_total == 26 else 'C5-style'}: ONE Twist::prove of a 2^{log_total}-op trace "
                    f"(src/benchmarks.rs:88-99) sharded over {world} GPUs (2^{log_total - (world.bit_length() - 1)} "
                    f"ops each), setup_params_shard({L}), slices resident in HBM")
        parallelism = f"one proof sharded x{world} ({args.comm} allgather of partial sums)"
    else:
        name = "C5 on one GPU" if log_total == 26 else ("C4" if log_total == 24 else f"2^{log_total} ops")
        workload = f"{name}: Twist::prove, 2^{log_total}-op trace, setup_params({L}), trace resident in HBM"
        parallelism = f"independent traces x{world}" if world > 1 else "single GPU"
    scaling = "weak" if (args.weak or args.independent) else "strong"

    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "ops/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt_max / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": scaling, "vs_baseline": None, "dtype": "u256 (8x u32 Montgomery, BN254 Fr/Fq)",
        "data": "synthetic (src/benchmarks.rs:88-99 trace)",
        "config": {"workload": workload, "log_ops": log_total, "ops_per_gpu": n_ops, "ops_per_proof": n_total,
                   "parallelism": parallelism,
                   "scaling_note": "N = 1 proves C4 (the metric's single-GPU config); N > 1 prove ONE C5 trace "
                                   "(2^26 ops, total fixed: strong scaling); --strong proves C5 at N = 1 too, "
                                   "--weak keeps 2^24 ops per GPU"},
        "comm": comm_cfg,
        "twist_last_prove_ms": {k: round(v, 3) for k, v in breakdown.items()},
        "commit_basis": args.commit_basis,
        "setup_ms": {"setup_params": round(t_setup * 1e3, 1), "lagrange_basis": round(t_lag * 1e3, 1)},
        "device_state": dstate.record(),
    }
    if rank == 0 and world == 1 and not args.no_extras:
        # drop-in rate: Twist::prove on host buffers through the C ABI (PCIe and host-side SoA
        # included), the same number of steps (SURVEY 8(d) measures prove() on host data); the
        # raw proof struct is what a Rust binding receives, so the Python mirror's proof objects
        # (Twist.prove_soa, ~0.7 ms of int conversions) stay out, as they do for `value`
        k = args.dropin_steps if args.dropin_steps is not None else args.steps
        if k > 0:
            t_di = timed_proofs(lambda: ts.twist_prove_host_raw(pp, addr, val, isw), k, 1)
            out["twist_ops_per_sec_dropin"] = round(n_ops / t_di, 2)
            out["ms_per_step_dropin"] = round(t_di * 1e3, 3)
            out["dropin_steps"] = k
        # the coefficient route (interpolation + coefficient KZG): an SRS without tau takes it
        if args.coef_steps > 0 and args.commit_basis == "lagrange":
            ctx.set_commit_basis(False)
            try:
                t_cf = timed_proofs(prove, args.coef_steps, 1)
            finally:
                ctx.set_commit_basis(True)
            out["twist_ops_per_sec_coefficient_route"] = round(n_ops / t_cf, 2)
            out["ms_per_step_coefficient_route"] = round(t_cf * 1e3, 3)
        # C2: MSM 2^20 pairs (setup_params(18)); scalars = Fr::rand from ChaCha20Rng([7;32])
        pp18, _ = ts.setup_params(18, device=local)
        if args.commit_basis == "lagrange":
            pp18.commitment_params.srs.prepare_lagrange(1 << 20)
        n = 1 << 20
        sc = ts.DeviceBuffer(ctx, ts.fr_rand_batch(bytes([7] * 32), n))
        t_msm = timed_proofs(lambda: ts.msm_resident(pp18.commitment_params, sc, n), 10, 1)
        out["msm_pairs_per_sec_2^20"] = round(n / t_msm, 1)
        out["msm_ms_2^20"] = round(t_msm * 1e3, 3)
        # the same commitment with no precomputation at all (the reference's commit,
        # src/commitments.rs:173-177, has none): variable-base Pippenger, per-window buckets
        ref = ts.msm_resident(pp18.commitment_params, sc, n)
        ctx.set_msm_tables(False)
        try:
            t_var = timed_proofs(lambda: ts.msm_resident(pp18.commitment_params, sc, n), 10, 1)
            same = bool((ts.msm_resident(pp18.commitment_params, sc, n) == ref).all())
        finally:
            ctx.set_msm_tables(not args.no_msm_tables)
        out["msm_pairs_per_sec_2^20_no_table"] = round(n / t_var, 1)
        out["msm_ms_2^20_no_table"] = round(t_var * 1e3, 3)
        out["msm_2^20_no_table_same_commitment"] = same
        out["msm_2^20_table_note"] = ("msm_*_2^20: fixed-base window table over the SRS (built once at setup, "
                                      "T[j n + i] = 2^(c j) g1_powers[i]); *_no_table: variable-base, no precomputation")
        # C4 with no window tables: the reference's commit has no precomputation
        # (src/commitments.rs:173-177); every MSM of the step runs per-window buckets over the
        # Lagrange basis itself, and the proof must be the one the table plans gave
        if args.no_table_steps > 0 and not args.no_msm_tables:
            want = bytes(prove())
            ctx.set_msm_tables(False)
            try:
                t_nt = timed_proofs(prove, args.no_table_steps, 1)
                same_nt = bytes(prove()) == want
            finally:
                ctx.set_msm_tables(True)
            out["ms_per_step_no_table"] = round(t_nt * 1e3, 3)
            out["twist_ops_per_sec_no_table"] = round(n_ops / t_nt, 2)
            out["no_table_steps"] = args.no_table_steps
            out["no_table_same_proof"] = same_nt
        # C3: Shout, 2^20 squares table, 2^20 lookups i % 2^20 (src/benchmarks.rs:167-177)
        T = 1 << 20
        entries = ts.fr_from_u64_array(np.arange(T, dtype=np.uint64) ** 2)
        idx = np.arange(T, dtype=np.uint64)
        d_e, d_i = ts.DeviceBuffer(ctx, entries), ts.DeviceBuffer(ctx, idx)
        t_sh = timed_proofs(lambda: ts.shout_prove_resident(pp18, d_e, T, d_i, T), 5, 1)
        out["shout_lookups_per_sec_2^20"] = round(T / t_sh, 1)
        out["shout_ms_2^20"] = round(t_sh * 1e3, 3)
    if rank == 0 and world == 1 and not args.no_extras and args.c5_steps > 0 and log_total == 24:
        out["c5_one_gpu"] = c5_one_gpu(ts, ctx, local, args.c5_steps)
        out["c5_one_gpu_ms_per_step"] = out["c5_one_gpu"].get("ms_per_step")
    if sharded and not args.no_extras:  # the MSM half of the metric at N GPUs (C2 sharded)
        with exchange_guard(ts, rank, "KZG MSM 2^20 (sharded)"):
            out.update(sharded_msm(ts, ctx, comm, pg, local, rank, world))
    if rank == 0 and world == 1 and not args.no_extras and args.tau_free_log > 0:
        out["tau_free_route"] = tau_free_route(ts, ctx, args.tau_free_log)
    if rank == 0 and world == 1 and not args.no_extras and args.sumcheck_logs:
        out["sumcheck_generic"] = sumcheck_generic(ts, ctx, [int(x) for x in args.sumcheck_logs.split(",")])
    if roof is not None:
        out["roofline"] = roof
        out["stages_ms_per_step"] = {k: round(v["ms"] / stage_steps, 3) for k, v in stages.items()}
        out["stages_timed_on"] = ("the timed steps" if args.profile_all_timed or args.stage_steps <= 0
                                  else f"{stage_steps} untimed steps after the timed region")
    if rank == 0 and world == 1 and not args.no_extras:
        out["cpu_baseline"] = cpu_baseline(ts, ctx, args.cpu_fast_log_ops, args.cpu_threads, pp=pp)
        lo, hi = (int(x) for x in args.cpu_ref_logs.split("-"))
        out["cpu_reference_algorithms"] = cpu_reference_algorithms(range(lo, hi + 1))
    if rank == 0:
        print(json.dumps(out), flush=True)
    if pg is not None:
        pg.barrier()
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
