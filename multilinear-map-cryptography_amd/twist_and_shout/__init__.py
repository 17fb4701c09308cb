"""twist_and_shout -- MI355X-native prover hot path with the reference crate's API.

Host-side mirror of the Rust crate ``twist-and-shout`` (/root/reference/src/lib.rs:41-56)
over the C ABI of ``libtns.so`` (include/tns.h).  Names, argument meaning and error
behaviour follow the reference:

* ``setup_params(log_size)``                       -- src/utils.rs:79-131
* ``MemoryTrace`` / ``Twist.prove``                 -- src/twist.rs:24-252
* ``LookupTable`` / ``Shout.prove``                 -- src/shout.rs:26-222
* ``KZGCommitment.commit/open``, ``KZGCommitmentValue.hash`` -- src/commitments.rs:73-199
* ``MultilinearExtension``                          -- src/polynomials.rs:18-196
* ``SumCheck.prove``                                -- src/sumcheck.rs:56-110
* ``Transcript``                                    -- src/utils.rs:134-204
* ``poly_utils.lagrange_interpolate`` on nodes 0..n-1 -- src/polynomials.rs:301-352

Field elements are Python ints (canonical representatives mod r); bulk data is
passed to the device as uint64 (n, 4) Montgomery arrays (arkworks' memory layout).
Errors raise ``TwistAndShoutError`` subclasses named after the Rust enum variants
(src/lib.rs:59-78).
"""

from __future__ import annotations

import atexit
import ctypes as C
import threading
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _native as N

R_MOD = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001
P_MOD = 0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47
_MONT_R = 1 << 256
_MASK64 = (1 << 64) - 1

FieldElement = int
G1Affine = Optional[Tuple[int, int]]  # None = identity


# ----------------------------------------------------------------------------- errors
class TwistAndShoutError(Exception):
    """src/lib.rs:59-78"""


class InvalidParameters(TwistAndShoutError):
    pass


class ProofGeneration(TwistAndShoutError):
    pass


class ProofVerification(TwistAndShoutError):
    pass


class CommitmentError(TwistAndShoutError):
    pass


class PolynomialError(TwistAndShoutError):
    pass


class SumCheckError(TwistAndShoutError):
    pass


class DeviceError(TwistAndShoutError):
    pass


_ERRORS = {1: InvalidParameters, 2: ProofGeneration, 3: ProofVerification, 4: CommitmentError,
           5: PolynomialError, 6: SumCheckError}


def _check(status: int):
    if status != 0:
        raise _ERRORS.get(status, DeviceError)(f"[{N.STATUS_NAMES.get(status, status)}] {N.last_error()}")


# ----------------------------------------------------------------------------- conversions
def to_mont(values: Sequence[int], mod: int = R_MOD) -> np.ndarray:
    out = np.empty((len(values), 4), dtype=np.uint64)
    for i, v in enumerate(values):
        m = (int(v) % mod) * _MONT_R % mod
        out[i] = [(m >> 0) & _MASK64, (m >> 64) & _MASK64, (m >> 128) & _MASK64, (m >> 192) & _MASK64]
    return out


def _limbs_to_int(row) -> int:
    return int(row[0]) | int(row[1]) << 64 | int(row[2]) << 128 | int(row[3]) << 192


def from_mont(arr: np.ndarray, mod: int = R_MOD) -> List[int]:
    arr = np.ascontiguousarray(arr, dtype=np.uint64).reshape(-1, 4)
    canon = np.empty_like(arr)
    if len(arr):
        (N.load().tns_fr_to_canonical if mod == R_MOD else N.load().tns_fq_to_canonical)(
            N.p64(arr), len(arr), N.p64(canon))
    return [_limbs_to_int(r) for r in canon]


def fr_from_u64_array(vals: np.ndarray) -> np.ndarray:
    """Bulk Fr::from(u64) into Montgomery limbs (multi-threaded in libtns)."""
    v = np.ascontiguousarray(vals, dtype=np.uint64)
    out = np.empty((len(v), 4), dtype=np.uint64)
    if len(v):
        N.load().tns_fr_from_u64(N.p64(v), len(v), N.p64(out))
    return out


def _g1_from_proj(limbs) -> G1Affine:
    a = np.ascontiguousarray(np.asarray(limbs, dtype=np.uint64).reshape(3, 4))
    if not a[2].any():
        return None
    x, y = from_mont(a[:2], P_MOD)
    return (x, y)  # outputs are normalised with Z = 1


# ----------------------------------------------------------------------------- device context
_EXITING = False


def _mark_exiting():
    global _EXITING
    _EXITING = True


atexit.register(_mark_exiting)


class Context:
    """One libtns context (HIP stream + workspaces) per device and process."""

    _lock = threading.Lock()
    _by_device: dict = {}

    def __init__(self, device: int = 0, stream_priorities: bool = True):
        """stream_priorities=False (TNS_CTX_NO_STREAM_PRIORITIES): every stream at the default
        priority, for processes that share one GPU.  Same proofs."""
        lib = N.load()
        h = C.c_void_p()
        _check(lib.tns_ctx_create_ex(device, 0 if stream_priorities else 1, C.byref(h)))
        self.handle = h
        self.device = device
        self.stream_priorities = stream_priorities

    @classmethod
    def get(cls, device: int = 0, stream_priorities: bool = True) -> "Context":
        """The process's context on `device` (the first call creates it with `stream_priorities`)."""
        with cls._lock:
            if device not in cls._by_device:
                cls._by_device[device] = Context(device, stream_priorities)
            return cls._by_device[device]

    def __del__(self):
        # a private context (sharded ranks, tests) frees its streams and workspaces with its last
        # reference (its SRS objects and buffers hold one); never during interpreter shutdown,
        # when the HIP runtime may already be gone
        if _EXITING:
            return
        try:
            N.load().tns_ctx_destroy(self.handle)
        except Exception:
            pass

    def set_commit_basis(self, lagrange: bool):
        """True (default): Twist/Shout commit and open through the SRS's Lagrange basis
        when it has tau; False: vector_to_polynomial + coefficient KZG.  Same proofs."""
        _check(N.load().tns_ctx_set_commit_basis(self.handle, 1 if lagrange else 0))

    def set_upload_chunks(self, chunks: int):
        """Drop-in provers: the value vector crosses PCIe in `chunks` node ranges (1..64,
        default 4), each committed as it lands.  Same proofs."""
        _check(N.load().tns_ctx_set_upload_chunks(self.handle, int(chunks)))

    def set_msm_tables(self, on: bool):
        """True (default): MSMs over fixed bases use their window tables (one shared bucket
        set); False: per-window buckets.  Same results."""
        _check(N.load().tns_ctx_set_msm_tables(self.handle, 1 if on else 0))

    def timing(self):
        out = (C.c_double * 6)()
        N.load().tns_last_prove_timing(self.handle, out)
        return dict(zip(["h2d", "interpolate", "commit", "sumcheck", "open", "total"], list(out)))


def device_count() -> int:
    return N.load().tns_device_count()


def clock_probe(ctx: "Context", ms: float = 60.0) -> dict:
    """The shader clock held under a full VALU load of Montgomery products (tns_clock_probe):
    the in-kernel clock, median / min / max over workgroups, and the probe kernel's ms."""
    out = (C.c_double * 4)()
    _check(N.load().tns_clock_probe(ctx.handle, float(ms), out))
    return {"median_mhz": round(out[0], 1), "min_mhz": round(out[1], 1), "max_mhz": round(out[2], 1),
            "kernel_ms": round(out[3], 2)}


def device_info(device: int = 0) -> dict:
    """hipDeviceProp_t identity and clock ratings of one visible device (tns_device_info_get)."""
    info = N.TnsDeviceInfo()
    _check(N.load().tns_device_info_get(device, C.byref(info)))
    return {"name": info.name.decode(errors="replace"), "arch": info.arch.decode(errors="replace"),
            "pci_bus_id": info.pci_bus_id.decode(errors="replace"), "clock_khz": info.clock_khz,
            "mem_clock_khz": info.mem_clock_khz, "cu_count": info.cu_count, "total_mem": info.total_mem}


# ----------------------------------------------------------------------------- params
class Srs:
    """Device-resident CommitmentParams.g1_powers."""

    def __init__(self, ctx: Context, handle: C.c_void_p):
        self.ctx = ctx
        self.handle = handle

    def __len__(self):
        return N.load().tns_srs_len(self.handle)

    def set_tau(self, tau: int):
        """Attach the setup trapdoor (CommitmentParams.tau) so the Lagrange basis exists."""
        _check(N.load().tns_srs_set_tau(self.handle, N.p64(to_mont([tau]))))

    def prepare_lagrange_shard(self, n: int, rank: int, size: int):
        """Build rank's slice of the Lagrange basis for n nodes (sharded proving setup)."""
        _check(N.load().tns_srs_prepare_lagrange_shard(self.ctx.handle, self.handle, n, rank, size))

    def prepare_lagrange(self, n: int):
        """Build the Lagrange basis for n = 2^k nodes now (setup time) instead of at the
        first proof of that size."""
        _check(N.load().tns_srs_prepare_lagrange(self.ctx.handle, self.handle, n))

    def prepare_lagrange_from_powers(self, n: int):
        """Build the Lagrange basis for n = 2^k nodes from g1_powers alone (no tau needed): a
        one-time setup (tns_srs_prepare_lagrange_from_powers) after which provers on this SRS take
        the Lagrange route."""
        _check(N.load().tns_srs_prepare_lagrange_from_powers(self.ctx.handle, self.handle, n))

    def lagrange_points(self, n: int) -> np.ndarray:
        """The Lagrange basis [L_j(tau)]G of the nodes 0..n-1 (affine limbs, host copy)."""
        out = np.zeros((n, 8), dtype=np.uint64)
        _check(N.load().tns_srs_lagrange_download(self.ctx.handle, self.handle, n, N.p64(out)))
        return out

    def download(self, n: Optional[int] = None) -> np.ndarray:
        n = len(self) if n is None else n
        out = np.zeros((n, 8), dtype=np.uint64)
        _check(N.load().tns_srs_download(self.ctx.handle, self.handle, N.p64(out), n))
        return out

    def share(self) -> Tuple[int, int]:
        """(first, held): the slice of g1_powers this SRS holds (a shard's share, or all of it)."""
        a, b = C.c_uint64(), C.c_uint64()
        _check(N.load().tns_srs_share(self.handle, C.byref(a), C.byref(b)))
        return a.value, b.value

    def points_at(self, indices) -> np.ndarray:
        """g1_powers[i] for the given global indices (affine Montgomery limbs), within share()."""
        idx = np.ascontiguousarray(indices, dtype=np.uint64)
        out = np.zeros((len(idx), 8), dtype=np.uint64)
        if len(idx):
            _check(N.load().tns_srs_download_indices(self.ctx.handle, self.handle, N.p64(idx), len(idx),
                                                     N.p64(out)))
        return out

    def __del__(self):
        if _EXITING:  # the HIP runtime may already be gone (as Context.__del__)
            return
        try:
            N.load().tns_srs_destroy(self.handle)
        except Exception:
            pass


@dataclass
class CommitmentParams:
    """src/utils.rs:53-63 (g2_generator is verifier-side and not materialised here)."""
    srs: Srs
    tau: Optional[int]

    @property
    def g1_powers(self) -> List[G1Affine]:
        limbs = self.srs.download()
        xs = from_mont(limbs[:, :4], P_MOD)
        ys = from_mont(limbs[:, 4:], P_MOD)
        return [None if (x == 0 and y == 0) else (x, y) for x, y in zip(xs, ys)]

    @classmethod
    def from_g1_limbs(cls, limbs: np.ndarray, device: int = 0, tau=None) -> "CommitmentParams":
        """Upload g1_powers given as affine Montgomery limbs (n x 8 uint64, identity = zeros), e.g. an
        Srs.download(): an SRS without tau unless one is given."""
        ctx = Context.get(device)
        arr = np.ascontiguousarray(limbs, dtype=np.uint64).reshape(-1, 8)
        h = C.c_void_p()
        _check(N.load().tns_srs_upload(ctx.handle, N.p64(arr), len(arr), C.byref(h)))
        srs = Srs(ctx, h)
        if tau is not None:
            srs.set_tau(tau)
        return cls(srs, tau)

    @classmethod
    def from_g1_powers(cls, g1_powers: Sequence[G1Affine], device: int = 0, tau=None) -> "CommitmentParams":
        ctx = Context.get(device)
        flat = []
        for P in g1_powers:
            flat.append((0, 0) if P is None else P)
        arr = np.zeros((len(flat), 8), dtype=np.uint64)
        if flat:
            arr[:, :4] = to_mont([p[0] for p in flat], P_MOD)
            arr[:, 4:] = to_mont([p[1] for p in flat], P_MOD)
            for i, P in enumerate(g1_powers):
                if P is None:
                    arr[i] = 0
        h = C.c_void_p()
        _check(N.load().tns_srs_upload(ctx.handle, N.p64(arr), len(arr), C.byref(h)))
        srs = Srs(ctx, h)
        if tau is not None:
            srs.set_tau(tau)
        return cls(srs, tau)


@dataclass
class ProverParams:
    """src/utils.rs:21-34"""
    log_size: int
    max_operations: int
    commitment_params: CommitmentParams
    fiat_shamir_seed: bytes
    _raw: N.TnsParams = field(repr=False, default=None)

    def raw(self) -> N.TnsParams:
        if self._raw is None:
            r = N.TnsParams()
            r.log_size = self.log_size
            r.max_operations = self.max_operations
            r.num_powers = len(self.commitment_params.srs)
            r.fiat_shamir_seed = (C.c_uint8 * 32)(*self.fiat_shamir_seed)
            self._raw = r
        return self._raw


@dataclass
class CommitmentVerificationKey:
    """src/utils.rs:64-75: G1 generator, G2 generator, [tau]_2 (host-side pairing verifier)."""
    raw: N.TnsVk = field(repr=False)

    @staticmethod
    def from_tau(tau: int) -> "CommitmentVerificationKey":
        r = N.TnsParams()
        r.tau = (C.c_uint64 * 4)(*to_mont([tau])[0])
        vk = N.TnsVk()
        _check(N.load().tns_verifier_key(C.byref(r), C.byref(vk)))
        return CommitmentVerificationKey(vk)

    @staticmethod
    def _g2(limbs) -> Optional[Tuple[Tuple[int, int], Tuple[int, int]]]:
        a = np.ctypeslib.as_array(limbs).reshape(4, 4)
        if not a.any():
            return None
        v = from_mont(a, P_MOD)
        return ((v[0], v[1]), (v[2], v[3]))

    @property
    def g1_generator(self) -> G1Affine:
        a = np.ctypeslib.as_array(self.raw.g1).reshape(2, 4)
        x, y = from_mont(a, P_MOD)
        return (x, y)

    @property
    def g2_generator(self):
        return self._g2(self.raw.g2)

    @property
    def g2_tau(self):
        return self._g2(self.raw.g2_tau)


@dataclass
class VerifierParams:
    """src/utils.rs:37-50"""
    log_size: int
    max_operations: int
    fiat_shamir_seed: bytes
    commitment_vk: Optional[CommitmentVerificationKey] = None


def setup_params(log_size: int, device: int = 0) -> Tuple[ProverParams, VerifierParams]:
    """src/utils.rs:79-131 -- tau and the FS seed from ChaCha20Rng([42;32]); SRS on the GPU."""
    ctx = Context.get(device)
    raw = N.TnsParams()
    h = C.c_void_p()
    _check(N.load().tns_setup_params(ctx.handle, log_size, C.byref(raw), C.byref(h)))
    tau = from_mont(np.array(list(raw.tau), dtype=np.uint64))[0]
    seed = bytes(raw.fiat_shamir_seed)
    cp = CommitmentParams(Srs(ctx, h), tau)
    pp = ProverParams(int(raw.log_size), int(raw.max_operations), cp, seed, raw)
    vk = CommitmentVerificationKey.from_tau(tau)
    return pp, VerifierParams(int(raw.log_size), int(raw.max_operations), seed, vk)


# ----------------------------------------------------------------------------- transcript
_TERMS_CACHE: dict = {}  # SumCheck._terms: composition -> its C array (read-only for the library)


class Transcript:
    """src/utils.rs:134-204 (host side; the same code drives the device prover)."""

    def __init__(self, seed: bytes = bytes(32)):
        self._lib = N.load()
        self._h = self._lib.tns_transcript_new((C.c_uint8 * 32).from_buffer_copy(bytes(seed)))

    def __del__(self):
        try:
            self._lib.tns_transcript_free(self._h)
        except Exception:
            pass

    @staticmethod
    def _lab(label: bytes):
        return (C.c_uint8 * max(1, len(label))).from_buffer_copy(label or b"\0"), len(label)

    def append_field_element(self, label: bytes, x: int):
        lab, n = self._lab(label)
        a = to_mont([x])
        N.load().tns_transcript_append_field_element(self._h, lab, n, N.p64(a))

    def append_field_elements(self, label: bytes, xs: Sequence[int]):
        lab, n = self._lab(label)
        a = to_mont(list(xs)) if len(xs) else np.zeros((1, 4), dtype=np.uint64)
        N.load().tns_transcript_append_field_elements(self._h, lab, n, N.p64(a), len(xs))

    def challenge_field_element(self, label: bytes) -> int:
        lab, n = self._lab(label)
        out = np.zeros(4, dtype=np.uint64)
        N.load().tns_transcript_challenge_field_element(self._h, lab, n, N.p64(out))
        return from_mont(out)[0]

    def challenge_field_elements(self, label: bytes, count: int) -> List[int]:
        return [self.challenge_field_element(label + b"_" + str(i).encode()) for i in range(count)]


# ----------------------------------------------------------------------------- KZG
@dataclass
class KZGCommitmentValue:
    """src/commitments.rs:67-85"""
    commitment: G1Affine
    _proj: np.ndarray = field(repr=False, default=None, compare=False)

    def serialize(self, compressed: bool = True) -> bytes:
        return g1_serialize(self.commitment, compressed)

    @staticmethod
    def deserialize(data: bytes, compressed: bool = True) -> "KZGCommitmentValue":
        return KZGCommitmentValue(g1_deserialize(data, compressed))

    def hash(self) -> int:
        out = np.zeros(4, dtype=np.uint64)
        proj = self._proj if self._proj is not None else _affine_to_proj(self.commitment)
        _check(N.load().tns_commitment_hash(N.p64(np.ascontiguousarray(proj)), N.p64(out)))
        return from_mont(out)[0]


@dataclass
class KZGProof:
    """src/commitments.rs:89-91"""
    proof: G1Affine

    def serialize(self, compressed: bool = True) -> bytes:
        return g1_serialize(self.proof, compressed)

    @staticmethod
    def deserialize(data: bytes, compressed: bool = True) -> "KZGProof":
        return KZGProof(g1_deserialize(data, compressed))


def g1_serialize(P: G1Affine, compressed: bool = True) -> bytes:
    """ark-serialize 0.4 encoding of a G1 point (src/commitments.rs:94-154)."""
    out = (C.c_uint8 * (32 if compressed else 64))()
    _check(N.load().tns_g1_serialize(N.p64(_affine_to_proj(P)), 1 if compressed else 0, out))
    return bytes(out)


def g1_deserialize(data: bytes, compressed: bool = True) -> G1Affine:
    buf = (C.c_uint8 * len(data)).from_buffer_copy(data)
    proj = np.zeros(12, dtype=np.uint64)
    _check(N.load().tns_g1_deserialize(buf, 1 if compressed else 0, N.p64(proj)))
    return _g1_from_proj(proj)


def _affine_to_proj(P: G1Affine) -> np.ndarray:
    if P is None:
        one = to_mont([1], P_MOD)[0]
        return np.concatenate([one, one, np.zeros(4, dtype=np.uint64)])
    return np.concatenate([to_mont([P[0]], P_MOD)[0], to_mont([P[1]], P_MOD)[0], to_mont([1], P_MOD)[0]])


def _as_mont(poly) -> np.ndarray:
    if isinstance(poly, np.ndarray):
        return np.ascontiguousarray(poly, dtype=np.uint64).reshape(-1, 4)
    return to_mont(list(poly)) if len(poly) else np.zeros((0, 4), dtype=np.uint64)


def _nonempty(a: np.ndarray) -> np.ndarray:
    return a if len(a) else np.zeros((1, 4), dtype=np.uint64)


class KZGCommitment:
    """``impl CommitmentScheme for KZGCommitment`` (src/commitments.rs:156-302), prover half."""

    @staticmethod
    def commit(params: CommitmentParams, polynomial) -> KZGCommitmentValue:
        c = _as_mont(polynomial)
        out = np.zeros(12, dtype=np.uint64)
        _check(N.load().tns_kzg_commit(params.srs.ctx.handle, params.srs.handle, N.p64(_nonempty(c)), len(c),
                                       N.p64(out)))
        return KZGCommitmentValue(_g1_from_proj(out), out)

    @staticmethod
    def open(params: CommitmentParams, polynomial, point: int) -> Tuple[int, KZGProof]:
        c = _as_mont(polynomial)
        z = to_mont([point])[0]
        v = np.zeros(4, dtype=np.uint64)
        pi = np.zeros(12, dtype=np.uint64)
        _check(N.load().tns_kzg_open(params.srs.ctx.handle, params.srs.handle, N.p64(_nonempty(c)), len(c),
                                     N.p64(z), N.p64(v), N.p64(pi)))
        return from_mont(v)[0], KZGProof(_g1_from_proj(pi))


    @staticmethod
    def verify(vk: "CommitmentVerificationKey", commitment: KZGCommitmentValue, point: int, value: int,
               proof: KZGProof) -> bool:
        """src/commitments.rs:201-228: e(C - [v]_1, [1]_2) == e(pi, [tau]_2 - [z]_2)."""
        ok = C.c_int()
        _check(N.load().tns_kzg_verify(C.byref(vk.raw), N.p64(_affine_to_proj(commitment.commitment)),
                                       N.p64(to_mont([point])[0]), N.p64(to_mont([value])[0]),
                                       N.p64(_affine_to_proj(proof.proof)), C.byref(ok)))
        return bool(ok.value)

    @staticmethod
    def batch_verify(vk: "CommitmentVerificationKey", commitments, points, values, proofs) -> bool:
        """src/commitments.rs:230-301 (the reference's batched equation, as written)."""
        if not (len(commitments) == len(points) == len(values) == len(proofs)):
            raise CommitmentError("Batch verify input lengths must match")
        n = len(commitments)
        if n == 0:
            return True
        cs = np.concatenate([_affine_to_proj(c.commitment) for c in commitments])
        ps = np.concatenate([_affine_to_proj(p.proof) for p in proofs])
        ok = C.c_int()
        _check(N.load().tns_kzg_batch_verify(C.byref(vk.raw), n, N.p64(cs), N.p64(to_mont(list(points))),
                                             N.p64(to_mont(list(values))), N.p64(ps), C.byref(ok)))
        return bool(ok.value)

    @staticmethod
    def commit_evaluations(params: CommitmentParams, evaluations) -> KZGCommitmentValue:
        """commit(vector_to_polynomial(evaluations)) as Twist/Shout::prove do (len a power of two)."""
        y = _as_mont(evaluations)
        out = np.zeros(12, dtype=np.uint64)
        _check(N.load().tns_kzg_commit_evals(params.srs.ctx.handle, params.srs.handle, N.p64(_nonempty(y)),
                                             len(y), N.p64(out)))
        return KZGCommitmentValue(_g1_from_proj(out), out)

    @staticmethod
    def open_evaluations(params: CommitmentParams, evaluations, point: int) -> Tuple[int, KZGProof]:
        """open(vector_to_polynomial(evaluations), point) as Twist/Shout::prove do."""
        y = _as_mont(evaluations)
        z = to_mont([point])[0]
        v = np.zeros(4, dtype=np.uint64)
        pi = np.zeros(12, dtype=np.uint64)
        _check(N.load().tns_kzg_open_evals(params.srs.ctx.handle, params.srs.handle, N.p64(_nonempty(y)), len(y),
                                           N.p64(z), N.p64(v), N.p64(pi)))
        return from_mont(v)[0], KZGProof(_g1_from_proj(pi))


class KZGVectorCommitment:
    """``impl VectorCommitmentScheme for KZGVectorCommitment`` (src/commitments.rs:408-483):
    KZG over the interpolant of the vector on the nodes 0..n-1."""

    @staticmethod
    def commit(params: CommitmentParams, vector) -> KZGCommitmentValue:
        return KZGCommitment.commit_evaluations(params, vector)

    @staticmethod
    def open(params: CommitmentParams, vector, index: int) -> Tuple[int, KZGProof]:
        y = _as_mont(vector)
        v = np.zeros(4, dtype=np.uint64)
        pi = np.zeros(12, dtype=np.uint64)
        _check(N.load().tns_vc_open(params.srs.ctx.handle, params.srs.handle, N.p64(_nonempty(y)), len(y), index,
                                    N.p64(v), N.p64(pi)))
        return from_mont(v)[0], KZGProof(_g1_from_proj(pi))

    @staticmethod
    def verify(vk: "CommitmentVerificationKey", commitment: KZGCommitmentValue, index: int, value: int,
               proof: KZGProof) -> bool:
        return KZGCommitment.verify(vk, commitment, index, value, proof)


def msm(params: CommitmentParams, scalars) -> G1Affine:
    """Raw G1 MSM over the first len(scalars) SRS points (the commit kernel)."""
    c = _as_mont(scalars)
    out = np.zeros(12, dtype=np.uint64)
    _check(N.load().tns_msm(params.srs.ctx.handle, params.srs.handle, N.p64(_nonempty(c)), len(c), N.p64(out)))
    return _g1_from_proj(out)


# ----------------------------------------------------------------------------- polynomials
class poly_utils:  # noqa: N801  (mirrors the Rust module name)
    @staticmethod
    def interpolate_consecutive(values, device: int = 0) -> np.ndarray:
        """lagrange_interpolate over nodes (0..n-1); Montgomery array in, Montgomery array out."""
        y = _as_mont(values)
        out = np.zeros_like(y)
        if len(y):
            _check(N.load().tns_interpolate_consecutive(Context.get(device).handle, N.p64(y), len(y), N.p64(out)))
        return out

    @staticmethod
    def lagrange_interpolate(points: Sequence[Tuple[int, int]], device: int = 0) -> List[int]:
        """src/polynomials.rs:301-352 for the node set the prover uses (x_i = i, n a power of two)."""
        n = len(points)
        if n == 0:
            return []
        if any(int(x) % R_MOD != i for i, (x, _) in enumerate(points)) or (n & (n - 1)):
            raise PolynomialError("device interpolation supports the nodes 0..n-1 with n a power of two")
        return from_mont(poly_utils.interpolate_consecutive([y for _, y in points], device))

    @staticmethod
    def evaluate_polynomial(coeffs: Sequence[int], point: int) -> int:
        """src/polynomials.rs:355-357 (Horner; host)."""
        acc = 0
        for c in reversed(coeffs):
            acc = (acc * point + c) % R_MOD
        return acc


class MultilinearExtension:
    """src/polynomials.rs:18-196 -- evaluate / partial_evaluate run on the GPU (fold kernels)."""

    def __init__(self, num_vars: int, evaluations: Sequence[int]):
        self.num_vars = num_vars
        self.evaluations = [int(e) % R_MOD for e in evaluations]

    @classmethod
    def from_evaluations(cls, evaluations):  # :28-37
        n = len(evaluations)
        nv = max(n.bit_length() - 1, 0)
        if (1 << nv) != n:
            raise AssertionError("Evaluation vector length must be a power of 2")
        return cls(nv, evaluations)

    @classmethod
    def from_evaluations_vec(cls, num_vars: int, evaluations):  # :40-50
        size = 1 << num_vars
        e = list(evaluations)[:size]
        return cls(num_vars, e + [0] * (size - len(e)))

    @classmethod
    def from_sparse(cls, num_vars: int, entries):  # :54-67
        ev = [0] * (1 << num_vars)
        for i, v in entries:
            if i >= len(ev):
                raise AssertionError(f"Index {i} out of bounds for size {len(ev)}")
            ev[i] = v
        return cls(num_vars, ev)

    @classmethod
    def one_hot(cls, num_vars: int, index: int):  # :71-82
        if index >= (1 << num_vars):
            raise AssertionError("Index out of bounds")
        ev = [0] * (1 << num_vars)
        ev[index] = 1
        return cls(num_vars, ev)

    def _table(self) -> np.ndarray:
        """The evaluations as the device table: at most 2^num_vars entries (the C side
        zero-fills the rest).  The reference struct may hold any number of entries; its basis
        reads only the low num_vars index bits (:108-122), so entry i counts at i mod 2^nv."""
        size = 1 << self.num_vars
        ev = self.evaluations
        if len(ev) > size:
            folded = [0] * size
            for i, e in enumerate(ev):
                folded[i & (size - 1)] = (folded[i & (size - 1)] + e) % R_MOD
            ev = folded
        return _nonempty(to_mont(ev) if ev else np.zeros((0, 4), dtype=np.uint64))

    def evaluate(self, point: Sequence[int], device: int = 0) -> int:  # :85-103
        if len(point) != self.num_vars:
            raise AssertionError("Point dimension must match number of variables")
        ev = self._table()
        pt = _nonempty(to_mont(list(point)))
        out = np.zeros(4, dtype=np.uint64)
        _check(N.load().tns_mle_evaluate(Context.get(device).handle, N.p64(ev), min(len(self.evaluations), 1 << self.num_vars),
                                         self.num_vars, N.p64(pt), N.p64(out)))
        return from_mont(out)[0]

    def partial_evaluate(self, fixed: Sequence[int], device: int = 0) -> "MultilinearExtension":  # :126-161
        k = len(fixed)
        if k > self.num_vars:
            raise AssertionError("Cannot fix more variables than available")
        if k == 0:
            return MultilinearExtension(self.num_vars, list(self.evaluations))
        ev = self._table()
        fx = to_mont(list(fixed))
        out = np.zeros((1 << (self.num_vars - k), 4), dtype=np.uint64)
        _check(N.load().tns_mle_partial_evaluate(Context.get(device).handle, N.p64(ev),
                                                 min(len(self.evaluations), 1 << self.num_vars), self.num_vars,
                                                 N.p64(fx), k, N.p64(out)))
        return MultilinearExtension(self.num_vars - k, from_mont(out))

    def add(self, other: "MultilinearExtension") -> "MultilinearExtension":  # :164-177
        assert self.num_vars == other.num_vars, "Number of variables must match"
        return MultilinearExtension(self.num_vars, [(a + b) % R_MOD for a, b in zip(self.evaluations, other.evaluations)])

    def scalar_mul(self, s: int) -> "MultilinearExtension":  # :180-190
        return MultilinearExtension(self.num_vars, [a * s % R_MOD for a in self.evaluations])

    def sum_evaluations(self) -> int:  # :193-195
        return sum(self.evaluations) % R_MOD


# ----------------------------------------------------------------------------- sum-check
@dataclass
class SumCheckProof:
    """src/sumcheck.rs:25-31"""
    round_polynomials: List[List[int]]
    final_evaluation: int


class SumCheck:
    """src/sumcheck.rs:15-110.  The closure is an MLE composition
    sum_t coeff_t * prod_j tables[idx_tj] (each term of degree <= 3)."""

    def __init__(self, num_vars: int, claimed_sum: int):
        self.num_vars = num_vars
        self.claimed_sum = claimed_sum % R_MOD

    def prove(self, tables: Sequence[Sequence[int]], terms: Sequence[Tuple[int, Sequence[int]]],
              transcript: Transcript, device: int = 0, return_challenges: bool = False):
        nv = self.num_vars
        arrs = [np.ascontiguousarray(t if isinstance(t, np.ndarray) else to_mont(list(t)), dtype=np.uint64)
                for t in tables]
        for a in arrs:
            if len(a) != (1 << nv):
                raise InvalidParameters("every table needs 2^num_vars entries")
        ptrs = (N.U64P * max(1, len(arrs)))(*[N.p64(a) for a in arrs])
        tt = (N.TnsTerm * max(1, len(terms)))()
        for i, (coef, idx) in enumerate(terms):
            tt[i].coeff = (C.c_uint64 * 4)(*[int(x) for x in to_mont([coef])[0]])
            ix = list(idx) + [-1] * (3 - len(idx))
            tt[i].tables = (C.c_int32 * 3)(*ix)
        cl = to_mont([self.claimed_sum])[0]
        rounds = np.zeros((max(1, nv), 4, 4), dtype=np.uint64)
        fin = np.zeros(4, dtype=np.uint64)
        ch = np.zeros((max(1, nv), 4), dtype=np.uint64)
        _check(N.load().tns_sumcheck_prove(Context.get(device).handle, ptrs, len(arrs), nv, N.p64(cl), tt,
                                           len(terms), transcript._h, N.p64(rounds), N.p64(fin), N.p64(ch)))
        proof = SumCheckProof([from_mont(r) for r in rounds[:nv]], from_mont(fin)[0])
        if return_challenges:
            return proof, from_mont(ch[:nv]) if nv else []
        return proof

    @staticmethod
    def _terms(terms):
        # (a composition's C array is built once: the conversions cost ~30 us a call)
        key = tuple((int(coef), tuple(int(j) for j in idx)) for coef, idx in terms)
        tt = _TERMS_CACHE.get(key)
        if tt is None:
            tt = (N.TnsTerm * max(1, len(terms)))()
            for i, (coef, idx) in enumerate(key):
                tt[i].coeff = (C.c_uint64 * 4)(*[int(x) for x in to_mont([coef])[0]])
                tt[i].tables = (C.c_int32 * 3)(*(list(idx) + [-1] * (3 - len(idx))))
            if len(_TERMS_CACHE) < 64:
                _TERMS_CACHE[key] = tt
        return tt

    @staticmethod
    def composition_sum_resident(num_vars: int, tables: Sequence["DeviceBuffer"],
                                 terms: Sequence[Tuple[int, Sequence[int]]]) -> int:
        """sum over {0,1}^num_vars of the composition on device tables (the honest claimed sum)."""
        ptrs = (C.c_void_p * len(tables))(*[t.ptr for t in tables])
        out = np.zeros(4, dtype=np.uint64)
        _check(N.load().tns_composition_sum_device(tables[0].ctx.handle, ptrs, len(tables), num_vars,
                                                   SumCheck._terms(terms), len(terms), N.p64(out)))
        return from_mont(out)[0]

    def prove_resident(self, tables: Sequence["DeviceBuffer"], terms: Sequence[Tuple[int, Sequence[int]]],
                       transcript: Transcript, raw: bool = False):
        """The same proof on tables already resident in HBM (DeviceBuffers of 2^num_vars
        Montgomery Fr, only read).  raw=True returns the Montgomery arrays (rounds, final,
        challenges) without converting them (timing loops)."""
        nv = self.num_vars
        if not tables:
            raise InvalidParameters("no tables")
        ctx = tables[0].ctx
        for t in tables:
            if t.nbytes != 32 << nv:
                raise InvalidParameters("every table needs 2^num_vars entries")
        ptrs = (C.c_void_p * len(tables))(*[t.ptr for t in tables])
        cl = to_mont([self.claimed_sum])[0]
        rounds = np.zeros((max(1, nv), 4, 4), dtype=np.uint64)
        fin = np.zeros(4, dtype=np.uint64)
        ch = np.zeros((max(1, nv), 4), dtype=np.uint64)
        _check(N.load().tns_sumcheck_prove_device(ctx.handle, ptrs, len(tables), nv, N.p64(cl), self._terms(terms),
                                                  len(terms), transcript._h, N.p64(rounds), N.p64(fin), N.p64(ch)))
        if raw:
            return rounds[:nv], fin, ch[:nv]
        return SumCheckProof([from_mont(r) for r in rounds[:nv]], from_mont(fin)[0]), (from_mont(ch[:nv]) if nv else [])


# ----------------------------------------------------------------------------- Twist
@dataclass(frozen=True)
class MemoryOp:
    """src/twist.rs:17-20 (kind is "Read" or "Write")."""
    kind: str
    address: int
    value: int


class MemoryTrace:
    """src/twist.rs:24-72"""

    def __init__(self, memory_size: int):
        if memory_size <= 0 or memory_size & (memory_size - 1):
            raise AssertionError("Memory size must be power of 2")
        self.memory_size = memory_size
        self.operations: List[MemoryOp] = []
        self._memory = [0] * memory_size

    def write(self, address: int, value: int):
        if address >= self.memory_size:
            raise InvalidParameters("Address out of bounds")
        self._memory[address] = value % R_MOD
        self.operations.append(MemoryOp("Write", address, value % R_MOD))

    def read(self, address: int) -> int:
        if address >= self.memory_size:
            raise InvalidParameters("Address out of bounds")
        v = self._memory[address]
        self.operations.append(MemoryOp("Read", address, v))
        return v

    def soa(self):
        """(addr u64[n], value Montgomery (n,4), is_write u8[n]) -- the C-ABI layout."""
        ops = self.operations
        addr = np.array([o.address for o in ops], dtype=np.uint64)
        val = to_mont([o.value for o in ops]) if ops else np.zeros((0, 4), dtype=np.uint64)
        isw = np.array([1 if o.kind == "Write" else 0 for o in ops], dtype=np.uint8)
        return addr, val, isw


@dataclass
class TwistProof:
    """src/twist.rs:76-89 (+ diagnostics the reference computes but drops)."""
    address_commitment: KZGCommitmentValue
    value_commitment: KZGCommitmentValue
    consistency_proof: SumCheckProof
    opening_proofs: List[KZGProof]
    final_evaluations: List[int]
    opening_point: Optional[int] = None
    sumcheck_challenges: List[int] = field(default_factory=list)
    final_mle_evals: List[int] = field(default_factory=list)

    def serialize(self, compressed: bool = True) -> bytes:
        """Wire format: fields in declaration order (src/twist.rs:76-89), Vec = u64 length + items."""
        return _serialize_raw(_pack_proof(
            [self.address_commitment.commitment, self.value_commitment.commitment],
            self.consistency_proof.round_polynomials, self.consistency_proof.final_evaluation,
            [p.proof for p in self.opening_proofs], self.final_evaluations), compressed)

    @staticmethod
    def deserialize(data: bytes, compressed: bool = True) -> "TwistProof":
        u = _unpack_proof(_deserialize_raw(data, compressed), 3)
        return TwistProof(u["comms"][0], u["comms"][1], u["sc"], u["openings"], u["finals"])


def _pack_proof(commitments, rounds, final_eval, openings, finals, verify: bool = False) -> N.TnsProof:
    """Proof fields (affine points / ints) -> the C proof struct.

    verify=True follows Twist/Shout::verify (src/twist.rs:276, src/shout.rs:245): the openings
    are checked only when there are at least two opening proofs AND two final evaluations,
    and then only the first two of each; otherwise they are skipped.  For serialisation the
    proof must hold exactly 0 or 2 of each (the wire format's Vec lengths).  Round
    polynomials have the 4 coefficients the prover emits (src/sumcheck.rs:201-206) and there
    are at most TNS_MAX_ROUNDS of them."""
    if len(rounds) > N.TNS_MAX_ROUNDS:
        raise InvalidParameters(f"more than {N.TNS_MAX_ROUNDS} sum-check rounds")
    for coeffs in rounds:
        if len(coeffs) != 4:
            raise InvalidParameters("a round polynomial must have 4 coefficients")
    if verify:
        n_open = 2 if min(len(openings), len(finals)) >= 2 else 0
    else:
        if len(openings) != len(finals) or len(openings) not in (0, 2):
            raise InvalidParameters("a proof holds 0 or 2 openings and as many final evaluations")
        n_open = len(openings)
    pr = N.TnsProof()
    for i, c in enumerate(commitments):
        pr.commitments[i] = (C.c_uint64 * 12)(*_affine_to_proj(c))
    pr.num_rounds = len(rounds)
    for r, coeffs in enumerate(rounds):
        m = to_mont(list(coeffs))
        for x in range(4):
            pr.round_polynomials[r][x] = (C.c_uint64 * 4)(*m[x])
    pr.final_evaluation = (C.c_uint64 * 4)(*to_mont([final_eval])[0])
    pr.num_openings = n_open
    for i in range(n_open):
        pr.opening_proofs[i] = (C.c_uint64 * 12)(*_affine_to_proj(openings[i]))
        pr.final_evaluations[i] = (C.c_uint64 * 4)(*to_mont([finals[i]])[0])
    return pr


def _serialize_raw(pr: N.TnsProof, compressed: bool) -> bytes:
    n = C.c_size_t()
    _check(N.load().tns_proof_serialize(C.byref(pr), 1 if compressed else 0, None, 0, C.byref(n)))
    buf = (C.c_uint8 * n.value)()
    _check(N.load().tns_proof_serialize(C.byref(pr), 1 if compressed else 0, buf, n.value, C.byref(n)))
    return bytes(buf)


def _deserialize_raw(data: bytes, compressed: bool) -> N.TnsProof:
    pr = N.TnsProof()
    buf = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
    _check(N.load().tns_proof_deserialize(buf, len(data), 1 if compressed else 0, C.byref(pr)))
    return pr


def _unpack_proof(pr: N.TnsProof, n_mles: int):
    """The C proof struct -> Python values: every Fr of the proof in ONE canonicalising call and
    every Fq in one more (a call per field element cost ~2 ms per proof at 24 rounds)."""
    nr, no = pr.num_rounds, pr.num_openings
    arr = np.ctypeslib.as_array
    rounds = arr(pr.round_polynomials)[:nr].reshape(-1, 4)
    fr_parts = [rounds, arr(pr.final_evaluation).reshape(-1, 4)]
    fr_parts += [arr(pr.final_evaluations[i]).reshape(-1, 4) for i in range(no)]
    fr_parts.append(arr(pr.opening_point).reshape(-1, 4))
    fr_parts.append(arr(pr.sumcheck_challenges)[:nr].reshape(-1, 4))
    fr_parts.append(arr(pr.final_mle_evals)[:n_mles].reshape(-1, 4) if nr else np.zeros((0, 4), dtype=np.uint64))
    fr = from_mont(np.concatenate(fr_parts))
    k = 0

    def take(m):
        nonlocal k
        out = fr[k:k + m]
        k += m
        return out

    rp = take(4 * nr)
    fin = take(1)[0]
    fe = take(no)
    z = take(1)[0]
    chals = take(nr)
    mle = take(n_mles if nr else 0)
    comms = [arr(pr.commitments[i]).copy() for i in range(2)]
    ops = [arr(pr.opening_proofs[i]).copy() for i in range(no)]
    pts = [np.asarray(c, dtype=np.uint64).reshape(3, 4) for c in comms + ops]
    xy = from_mont(np.concatenate([p[:2] for p in pts]), P_MOD)
    aff = [None if not p[2].any() else (xy[2 * i], xy[2 * i + 1]) for i, p in enumerate(pts)]  # Z = 1 or 0
    return dict(
        comms=[KZGCommitmentValue(aff[i], c) for i, c in enumerate(comms)],
        sc=SumCheckProof([rp[4 * r:4 * r + 4] for r in range(nr)], fin),
        openings=[KZGProof(aff[2 + i]) for i in range(no)],
        finals=fe,
        z=z if no else None,
        chals=chals if nr else [],
        mle=mle if nr else [],
    )


def _horner(coeffs: Sequence[int], x: int) -> int:
    """field_utils::horner_eval (src/utils.rs:217-221): sum_i c_i x^i, any length (0 for none)."""
    acc = 0
    for c in reversed(list(coeffs)):
        acc = (acc * x + c) % R_MOD
    return acc


def _verify_general(labels, commitments, rounds, final_eval, openings, finals, verifier_params) -> bool:
    """Twist/Shout::verify (src/twist.rs:255-304, src/shout.rs:225-274) with SumCheck::verify
    (src/sumcheck.rs:113-153) on the host, for proof shapes the C proof struct cannot hold: round
    polynomials of any length (each is hashed into the transcript as it stands) and any number of
    rounds.  Never raises on a malformed shape: it returns the reference's Ok(bool)."""
    t = Transcript(verifier_params.fiat_shamir_seed)
    t.append_field_element(labels[0], KZGCommitmentValue(commitments[0]).hash())
    t.append_field_element(labels[1], KZGCommitmentValue(commitments[1]).hash())
    claim = 0
    for r, g in enumerate(rounds):
        g = [int(c) % R_MOD for c in g]
        if (_horner(g, 0) + _horner(g, 1)) % R_MOD != claim:
            return False
        t.append_field_elements(b"sumcheck_round_%d" % r, g)
        claim = _horner(g, t.challenge_field_element(b"sumcheck_challenge_%d" % r))
    if claim != int(final_eval) % R_MOD:
        return False
    ch = t.challenge_field_elements(b"opening_challenges", len(rounds))
    if ch and len(openings) >= 2 and len(finals) >= 2:
        vk = verifier_params.commitment_vk
        for k in range(2):
            if not KZGCommitment.verify(vk, KZGCommitmentValue(commitments[k]), ch[0], finals[k], KZGProof(openings[k])):
                return False
    return True


def _c_struct_shape(rounds) -> bool:
    return len(rounds) <= N.TNS_MAX_ROUNDS and all(len(g) == 4 for g in rounds)


class Twist:
    """src/twist.rs:93-316 (prover)."""

    def __init__(self, prover_params: ProverParams):
        self.prover_params = prover_params

    def prove_soa(self, addr: np.ndarray, value: np.ndarray, is_write: np.ndarray) -> TwistProof:
        pp = self.prover_params
        srs = pp.commitment_params.srs
        addr = np.ascontiguousarray(addr, dtype=np.uint64)
        value = np.ascontiguousarray(value, dtype=np.uint64).reshape(-1, 4)
        is_write = np.ascontiguousarray(is_write, dtype=np.uint8)
        n = len(addr)
        pr = N.TnsProof()
        _check(N.load().tns_twist_prove(
            srs.ctx.handle, srs.handle, C.byref(pp.raw()),
            N.p64(addr if n else np.zeros(1, dtype=np.uint64)), N.p64(_nonempty(value)),
            N.p8(is_write if n else np.zeros(1, dtype=np.uint8)), n, C.byref(pr)))
        u = _unpack_proof(pr, 3)
        return TwistProof(u["comms"][0], u["comms"][1], u["sc"], u["openings"], u["finals"], u["z"], u["chals"],
                          u["mle"])

    def prove(self, trace: MemoryTrace) -> TwistProof:
        return self.prove_soa(*trace.soa())

    @staticmethod
    def verify(proof: TwistProof, verifier_params: VerifierParams) -> bool:
        """src/twist.rs:255-304 (host: sum-check replay + two pairing checks)."""
        comms = [proof.address_commitment.commitment, proof.value_commitment.commitment]
        if not _c_struct_shape(proof.consistency_proof.round_polynomials):
            return _verify_general((b"address_commitment", b"value_commitment"), comms,
                                   proof.consistency_proof.round_polynomials, proof.consistency_proof.final_evaluation,
                                   [p.proof for p in proof.opening_proofs], proof.final_evaluations, verifier_params)
        pr = _pack_proof([proof.address_commitment.commitment, proof.value_commitment.commitment],
                         proof.consistency_proof.round_polynomials, proof.consistency_proof.final_evaluation,
                         [p.proof for p in proof.opening_proofs], proof.final_evaluations, verify=True)
        ok = C.c_int()
        _check(N.load().tns_twist_verify(C.byref(verifier_params.commitment_vk.raw), C.byref(pr), C.byref(ok)))
        return bool(ok.value)

    def prove_sharded(self, comm: "Comm", addr: np.ndarray, value: np.ndarray, is_write: np.ndarray,
                      n_total: int) -> TwistProof:
        """This rank's slice (shard_slice(n_total, rank, size)) of one trace; every rank
        returns the same proof as the unsharded prove."""
        ctx = self.prover_params.commitment_params.srs.ctx
        n = len(addr)
        da = _nonempty_buf(ctx, addr, np.uint64)
        dv = _nonempty_buf(ctx, np.asarray(value, dtype=np.uint64).reshape(-1, 4), np.uint64, 4)
        dw = _nonempty_buf(ctx, is_write, np.uint8)
        return twist_proof_from_raw(twist_prove_sharded_resident(self.prover_params, comm, da, dv, dw, n, n_total))


# ----------------------------------------------------------------------------- Shout
@dataclass(frozen=True)
class LookupOp:
    """src/shout.rs:17-22"""
    index: int
    value: int


class LookupTable:
    """src/shout.rs:26-60"""

    def __init__(self, entries: Sequence[int]):
        self.entries = [int(e) % R_MOD for e in entries]
        self.lookups: List[LookupOp] = []

    def lookup(self, index: int) -> int:
        if index >= len(self.entries):
            raise InvalidParameters("Lookup index out of bounds")
        v = self.entries[index]
        self.lookups.append(LookupOp(index, v))
        return v

    def size(self) -> int:
        return len(self.entries)


@dataclass
class ShoutProof:
    """src/shout.rs:64-79"""
    table_commitment: KZGCommitmentValue
    index_commitment: KZGCommitmentValue
    lookup_proof: SumCheckProof
    opening_proofs: List[KZGProof]
    final_evaluations: List[int]
    opening_point: Optional[int] = None
    sumcheck_challenges: List[int] = field(default_factory=list)

    def serialize(self, compressed: bool = True) -> bytes:
        """Wire format: fields in declaration order (src/shout.rs:64-79)."""
        return _serialize_raw(_pack_proof(
            [self.table_commitment.commitment, self.index_commitment.commitment],
            self.lookup_proof.round_polynomials, self.lookup_proof.final_evaluation,
            [p.proof for p in self.opening_proofs], self.final_evaluations), compressed)

    @staticmethod
    def deserialize(data: bytes, compressed: bool = True) -> "ShoutProof":
        u = _unpack_proof(_deserialize_raw(data, compressed), 1)
        return ShoutProof(u["comms"][0], u["comms"][1], u["sc"], u["openings"], u["finals"])


class Shout:
    """src/shout.rs:83-286 (prover)."""

    def __init__(self, prover_params: ProverParams):
        self.prover_params = prover_params

    def prove_arrays(self, entries_mont: np.ndarray, indices: np.ndarray) -> ShoutProof:
        pp = self.prover_params
        srs = pp.commitment_params.srs
        e = np.ascontiguousarray(entries_mont, dtype=np.uint64).reshape(-1, 4)
        ix = np.ascontiguousarray(indices, dtype=np.uint64)
        pr = N.TnsProof()
        _check(N.load().tns_shout_prove(srs.ctx.handle, srs.handle, C.byref(pp.raw()), N.p64(_nonempty(e)), len(e),
                                        N.p64(ix if len(ix) else np.zeros(1, dtype=np.uint64)), len(ix),
                                        C.byref(pr)))
        u = _unpack_proof(pr, 1)
        return ShoutProof(u["comms"][0], u["comms"][1], u["sc"], u["openings"], u["finals"], u["z"], u["chals"])

    def prove_sharded(self, comm: "Comm", entries_mont: np.ndarray, n_entries_total: int, indices: np.ndarray,
                      n_lookups_total: int) -> ShoutProof:
        """This rank's slices of the table and of the lookup indices (shard_slice)."""
        ctx = self.prover_params.commitment_params.srs.ctx
        e = np.asarray(entries_mont, dtype=np.uint64).reshape(-1, 4)
        de = _nonempty_buf(ctx, e, np.uint64, 4)
        di = _nonempty_buf(ctx, indices, np.uint64)
        return shout_proof_from_raw(shout_prove_sharded_resident(self.prover_params, comm, de, len(e),
                                                                 n_entries_total, di, len(indices), n_lookups_total))

    @staticmethod
    def verify(proof: ShoutProof, verifier_params: VerifierParams) -> bool:
        """src/shout.rs:225-274"""
        comms = [proof.table_commitment.commitment, proof.index_commitment.commitment]
        if not _c_struct_shape(proof.lookup_proof.round_polynomials):
            return _verify_general((b"table_commitment", b"index_commitment"), comms,
                                   proof.lookup_proof.round_polynomials, proof.lookup_proof.final_evaluation,
                                   [p.proof for p in proof.opening_proofs], proof.final_evaluations, verifier_params)
        pr = _pack_proof([proof.table_commitment.commitment, proof.index_commitment.commitment],
                         proof.lookup_proof.round_polynomials, proof.lookup_proof.final_evaluation,
                         [p.proof for p in proof.opening_proofs], proof.final_evaluations, verify=True)
        ok = C.c_int()
        _check(N.load().tns_shout_verify(C.byref(verifier_params.commitment_vk.raw), C.byref(pr), C.byref(ok)))
        return bool(ok.value)

    def prove(self, table: LookupTable) -> ShoutProof:
        e = to_mont(table.entries) if table.entries else np.zeros((0, 4), dtype=np.uint64)
        ix = np.array([l.index for l in table.lookups], dtype=np.uint64)
        return self.prove_arrays(e, ix)


class DeviceBuffer:
    """An input array resident in HBM (tns_buffer_upload)."""

    def __init__(self, ctx: Context, host: np.ndarray):
        host = np.ascontiguousarray(host)
        self.ctx = ctx
        self.nbytes = host.nbytes
        self.handle = C.c_void_p()
        _check(N.load().tns_buffer_upload(ctx.handle, host.ctypes.data_as(C.c_void_p), host.nbytes,
                                          C.byref(self.handle)))
        self.ptr = N.load().tns_buffer_device_ptr(self.handle)

    def __del__(self):
        if _EXITING:
            return
        try:
            N.load().tns_buffer_free(self.handle)
        except Exception:
            pass


def buffer_download(buf: DeviceBuffer, out: np.ndarray):
    """Copy the buffer's first out.nbytes bytes into the (C-contiguous) host array out."""
    assert out.flags["C_CONTIGUOUS"]
    _check(N.load().tns_buffer_download(buf.handle, out.ctypes.data_as(C.c_void_p), out.nbytes))


def twist_prove_resident(pp: ProverParams, addr: DeviceBuffer, value: DeviceBuffer, is_write: DeviceBuffer,
                         n_ops: int) -> N.TnsProof:
    """Twist::prove on a trace already resident in HBM; returns the raw C proof struct."""
    srs = pp.commitment_params.srs
    pr = N.TnsProof()
    _check(N.load().tns_twist_prove_device(srs.ctx.handle, srs.handle, C.byref(pp.raw()), addr.ptr, value.ptr,
                                           is_write.ptr, n_ops, C.byref(pr)))
    return pr


def twist_prove_host_raw(pp: ProverParams, addr: np.ndarray, value: np.ndarray, is_write: np.ndarray) -> N.TnsProof:
    """Twist::prove on host buffers through the C ABI (tns_twist_prove: the drop-in call a Rust
    binding makes, PCIe included); returns the raw C proof struct -- what the Rust side receives --
    without building the Python proof objects (Twist.prove_soa adds those)."""
    srs = pp.commitment_params.srs
    addr = np.ascontiguousarray(addr, dtype=np.uint64)
    value = np.ascontiguousarray(value, dtype=np.uint64).reshape(-1, 4)
    is_write = np.ascontiguousarray(is_write, dtype=np.uint8)
    n = len(addr)
    pr = N.TnsProof()
    _check(N.load().tns_twist_prove(srs.ctx.handle, srs.handle, C.byref(pp.raw()),
                                    N.p64(addr if n else np.zeros(1, dtype=np.uint64)), N.p64(_nonempty(value)),
                                    N.p8(is_write if n else np.zeros(1, dtype=np.uint8)), n, C.byref(pr)))
    return pr


def shout_prove_resident(pp: ProverParams, entries: DeviceBuffer, n_entries: int, indices: DeviceBuffer,
                         n_lookups: int) -> N.TnsProof:
    srs = pp.commitment_params.srs
    pr = N.TnsProof()
    _check(N.load().tns_shout_prove_device(srs.ctx.handle, srs.handle, C.byref(pp.raw()), entries.ptr, n_entries,
                                           indices.ptr, n_lookups, C.byref(pr)))
    return pr


def msm_resident(params: CommitmentParams, scalars: DeviceBuffer, n: int) -> np.ndarray:
    out = np.zeros(12, dtype=np.uint64)
    _check(N.load().tns_msm_device(params.srs.ctx.handle, params.srs.handle, scalars.ptr, n, N.p64(out)))
    return out


# ----------------------------------------------------------------------------- one proof across GPUs
_AllgatherFn = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p)


class ExchangeTimeout(DeviceError):
    """An exchange step of a sharded proof passed its deadline (a peer rank stalled or died)."""


class Comm:
    """Communicator of one sharded proof (tns_comm): the allgathers of partial MSM sums,
    barycentric partials and folded table values.

    Every exchange step has a deadline (`timeout_s`, default 600 s): the RCCL transport polls its
    collective and aborts the communicator, a host-callback transport enforces it in the
    callback.  A step that misses it fails the prove call with a message naming this rank, the
    step number and what it carried -- and, for the torch transport, the last step every peer
    rank reached (from the process group's store), i.e. which rank stalled."""

    DEFAULT_TIMEOUT_S = 600.0

    def __init__(self, handle: C.c_void_p, rank: int, size: int, keep=None, timeout_s: Optional[float] = None):
        self.handle, self.rank, self.size, self._keep = handle, rank, size, keep
        self.last_failure: Optional[str] = None
        # a host-callback transport whose exchange failed (deadline, transport error) is dead: a
        # later exchange would pair with a peer's late collective, so it is refused (the RCCL
        # transport aborts its communicator likewise); tear the process group down to recover
        self.failed = False
        # None: the default deadline; 0 or less is the caller's error (tns_comm_set_timeout refuses it)
        self.timeout_s = self.DEFAULT_TIMEOUT_S if timeout_s is None else float(timeout_s)
        _check(N.load().tns_comm_set_timeout(self.handle, self.timeout_s))

    def set_timeout(self, seconds: float):
        _check(N.load().tns_comm_set_timeout(self.handle, float(seconds)))
        self.timeout_s = float(seconds)

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * 128)()
        _check(N.load().tns_comm_unique_id(buf))
        return bytes(buf)

    @classmethod
    def rccl(cls, ctx: Context, rank: int, size: int, uid: bytes, timeout_s: Optional[float] = None) -> "Comm":
        """RCCL communicator (ncclAllGather over xGMI); uid from Comm.unique_id() on rank 0."""
        h = C.c_void_p()
        _check(N.load().tns_comm_create(ctx.handle, rank, size, (C.c_uint8 * 128)(*uid), C.byref(h)))
        return cls(h, rank, size, timeout_s=timeout_s)

    @classmethod
    def from_allgather(cls, rank: int, size: int, fn, timeout_s: Optional[float] = None) -> "Comm":
        """fn(local: bytes) -> bytes: every rank's bytes concatenated in rank order.  fn may take
        a keyword `deadline_s` (the communicator's deadline) and should raise past it."""
        holder = {}

        def cb(user, send, nbytes, recv):
            me = holder.get("comm")
            if me is not None and me.failed:
                me.last_failure = ("this communicator failed at an earlier exchange (its collective may still be "
                                   "pending on a peer); tear the process group down and create a new one")
                return 4
            try:
                out = fn(C.string_at(send, nbytes), **({"deadline_s": me.timeout_s} if holder.get("kw") else {}))
                if len(out) != nbytes * size:
                    if me is not None:
                        me.last_failure = f"allgather returned {len(out)} bytes, expected {nbytes * size}"
                        me.failed = True
                    return 2
                C.memmove(recv, out, len(out))
                return 0
            except Exception as e:  # noqa: BLE001 -- reported to the library as a failed exchange
                if me is not None:
                    me.last_failure = f"{type(e).__name__}: {e}"
                    me.failed = True
                return 3 if isinstance(e, TimeoutError) else 1
        import inspect

        try:
            holder["kw"] = "deadline_s" in inspect.signature(fn).parameters
        except (TypeError, ValueError):
            holder["kw"] = False
        cfn = _AllgatherFn(cb)
        h = C.c_void_p()
        _check(N.load().tns_comm_create_callback(rank, size, C.cast(cfn, C.c_void_p), None, C.byref(h)))
        comm = cls(h, rank, size, keep=cfn, timeout_s=timeout_s)
        holder["comm"] = comm
        return comm

    @classmethod
    def torch(cls, group=None, device=None, timeout_s: Optional[float] = None) -> "Comm":
        """Allgather through an initialised torch.distributed process group (nccl = RCCL on
        ROCm, or gloo), with a deadline per step: the collective is issued asynchronously and
        polled; before it each rank publishes its step number in the group's store, so a rank
        whose step passes the deadline reports which peers never reached that step."""
        import torch
        import torch.distributed as dist

        rank, size = dist.get_rank(group), dist.get_world_size(group)
        try:
            from torch.distributed import distributed_c10d as c10d

            store = c10d._get_default_store()
        except Exception:  # noqa: BLE001 -- diagnostics only
            store = None
        state = {"step": 0}

        def peers_behind(step):
            if store is None:
                return "peer steps unknown (no process-group store)"
            seen = []
            for r in range(size):
                key = f"tns_comm/step/{r}"
                try:
                    v = int(store.get(key)) if store.check([key]) else 0
                except Exception:  # noqa: BLE001
                    v = -1
                seen.append(v)
            late = [r for r, v in enumerate(seen) if v < step]
            return f"peer ranks still before step {step}: {late} (last step per rank: {seen})"

        def fn(data: bytes, deadline_s: float = cls.DEFAULT_TIMEOUT_S) -> bytes:
            import time as _time

            state["step"] += 1
            step = state["step"]
            if store is not None:
                try:
                    store.set(f"tns_comm/step/{rank}", str(step))
                except Exception:  # noqa: BLE001
                    pass
            t = torch.frombuffer(bytearray(data), dtype=torch.uint8)
            if device is not None:
                t = t.to(device)
            out = torch.empty(len(data) * size, dtype=torch.uint8, device=t.device)
            work = dist.all_gather_into_tensor(out, t, group=group, async_op=True)
            t0 = _time.monotonic()
            while not work.is_completed():
                if _time.monotonic() - t0 > deadline_s:
                    raise TimeoutError(f"rank {rank}: allgather step {step} ({len(data)} B) passed its "
                                       f"{deadline_s:g} s deadline; {peers_behind(step)}")
                _time.sleep(0.0002)
            work.wait()
            return out.cpu().numpy().tobytes()
        return cls.from_allgather(rank, size, fn, timeout_s=timeout_s)

    KINDS = {0: "self", 1: "callback", 2: "rccl"}

    def info(self) -> dict:
        """rank, size, the rank count the transport reports (ncclCommCount for RCCL) and kind."""
        r, n, seen, k = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        _check(N.load().tns_comm_info(self.handle, C.byref(r), C.byref(n), C.byref(seen), C.byref(k)))
        return {"rank": r.value, "size": n.value, "seen_size": seen.value, "kind": self.KINDS.get(k.value, "?")}

    def stats(self) -> dict:
        """Exchange steps so far, their host-timed latency and this rank's bytes (tns_comm_stats_ex)."""
        out = (C.c_double * 6)()
        _check(N.load().tns_comm_stats_ex(self.handle, out))
        n = int(out[0])
        return {"exchanges": n, "total_s": out[1], "mean_us": (out[1] / n * 1e6) if n else None,
                "max_us": out[2] * 1e6 if n else None, "timeout_s": out[3], "bytes_total": out[4],
                "max_bytes": out[5] if n else None}

    def allgather(self, data: bytes, ctx: Optional[Context] = None) -> bytes:
        """The communicator's own allgather (every rank's bytes, in rank order)."""
        src = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
        out = (C.c_uint8 * max(1, len(data) * self.size))()
        self.check(N.load().tns_comm_allgather(ctx.handle if ctx else None, self.handle, src, len(data), out))
        return bytes(out)[:len(data) * self.size]

    def check(self, status: int):
        """_check for a call that exchanged through this communicator: a failed exchange step
        raises ExchangeTimeout (deadline) or DeviceError with the transport's own diagnosis."""
        if status == 0:
            return
        msg = f"[{N.STATUS_NAMES.get(status, status)}] {N.last_error()}"
        if self.last_failure:
            msg += f" -- {self.last_failure}"
        if "timed out" in msg or "deadline" in msg:
            raise ExchangeTimeout(msg)
        raise _ERRORS.get(status, DeviceError)(msg)

    def __del__(self):
        if _EXITING:  # interpreter shutdown: RCCL / HIP may already be torn down (as Context.__del__)
            return
        try:
            N.load().tns_comm_destroy(self.handle)
        except Exception:
            pass


def setup_params_shard(log_size: int, rank: int, size: int, device: int = 0,
                       ctx: Optional[Context] = None) -> Tuple[ProverParams, VerifierParams]:
    """setup_params for rank `rank` of `size`: same params and tau; the SRS holds only this
    rank's contiguous share of g1_powers."""
    ctx = ctx or Context.get(device)
    raw = N.TnsParams()
    h = C.c_void_p()
    _check(N.load().tns_setup_params_shard(ctx.handle, log_size, rank, size, C.byref(raw), C.byref(h)))
    tau = from_mont(np.array(list(raw.tau), dtype=np.uint64))[0]
    seed = bytes(raw.fiat_shamir_seed)
    cp = CommitmentParams(Srs(ctx, h), tau)
    pp = ProverParams(int(raw.log_size), int(raw.max_operations), cp, seed, raw)
    vk = CommitmentVerificationKey.from_tau(tau)
    return pp, VerifierParams(int(raw.log_size), int(raw.max_operations), seed, vk)


def shard_slice(n_total: int, rank: int, size: int) -> Tuple[int, int]:
    """(first, count) of rank's slice of an n_total-entry vector padded to a power of two."""
    L = (1 << max(0, (n_total - 1).bit_length())) // size
    first = rank * L
    return first, max(0, min(L, n_total - first))


def msm_sharded_resident(params: CommitmentParams, comm: Comm, scalars: DeviceBuffer, n_local: int,
                         n_total: int) -> np.ndarray:
    """KZGCommitment::commit of n_total coefficients sharded over comm's ranks (tns_msm_sharded):
    this rank's slice (shard_slice) resident in HBM, its SRS share from setup_params_shard.
    Returns the commitment's projective limbs (every rank the same)."""
    srs = params.srs
    out = np.zeros(12, dtype=np.uint64)
    comm.check(N.load().tns_msm_sharded(srs.ctx.handle, srs.handle, comm.handle, scalars.ptr, n_local, n_total,
                                    N.p64(out)))
    return out


def twist_prove_sharded_resident(pp: ProverParams, comm: Comm, addr: DeviceBuffer, value: DeviceBuffer,
                                 is_write: DeviceBuffer, n_local: int, n_total: int) -> N.TnsProof:
    srs = pp.commitment_params.srs
    pr = N.TnsProof()
    comm.check(N.load().tns_twist_prove_sharded(srs.ctx.handle, srs.handle, C.byref(pp.raw()), comm.handle, addr.ptr,
                                            value.ptr, is_write.ptr, n_local, n_total, C.byref(pr)))
    return pr


def shout_prove_sharded_resident(pp: ProverParams, comm: Comm, entries: DeviceBuffer, n_entries: int,
                                 n_entries_total: int, indices: DeviceBuffer, n_lookups: int,
                                 n_lookups_total: int) -> N.TnsProof:
    srs = pp.commitment_params.srs
    pr = N.TnsProof()
    comm.check(N.load().tns_shout_prove_sharded(srs.ctx.handle, srs.handle, C.byref(pp.raw()), comm.handle, entries.ptr,
                                            n_entries, n_entries_total, indices.ptr, n_lookups, n_lookups_total,
                                            C.byref(pr)))
    return pr


def twist_proof_from_raw(pr: N.TnsProof) -> "TwistProof":
    u = _unpack_proof(pr, 3)
    return TwistProof(u["comms"][0], u["comms"][1], u["sc"], u["openings"], u["finals"], u["z"], u["chals"], u["mle"])


def shout_proof_from_raw(pr: N.TnsProof) -> "ShoutProof":
    u = _unpack_proof(pr, 1)
    return ShoutProof(u["comms"][0], u["comms"][1], u["sc"], u["openings"], u["finals"], u["z"], u["chals"])


def _nonempty_buf(ctx: Context, a: np.ndarray, dtype, width: int = 1) -> DeviceBuffer:
    a = np.ascontiguousarray(a, dtype=dtype)
    if a.size == 0:
        a = np.zeros(width, dtype=dtype)
    return DeviceBuffer(ctx, a)


def bench_trace_slice(memory_size: int, n_total: int, first: int, count: int):
    """Operations [first, first + count) of the n_total-op ProtocolBenchmarks trace."""
    addr = np.empty(count, dtype=np.uint64)
    val = np.empty(count, dtype=np.uint64)
    isw = np.empty(count, dtype=np.uint8)
    if count:
        _check(N.load().tns_bench_trace_slice(memory_size, n_total, first, count, N.p64(addr), N.p64(val),
                                              N.p8(isw)))
    return addr, fr_from_u64_array(val), isw


def pairing(P: G1Affine, Q) -> List[int]:
    """Bn254::pairing(P, Q) -- 12 Fq coefficients (canonical) in the product's tower order."""
    g1 = np.zeros(8, dtype=np.uint64)
    if P is not None:
        g1[:4] = to_mont([P[0]], P_MOD)[0]
        g1[4:] = to_mont([P[1]], P_MOD)[0]
    g2 = np.zeros(16, dtype=np.uint64)
    if Q is not None:
        g2[:] = to_mont([Q[0][0], Q[0][1], Q[1][0], Q[1][1]], P_MOD).reshape(-1)
    out = np.zeros(48, dtype=np.uint64)
    _check(N.load().tns_pairing(N.p64(g1), N.p64(g2), N.p64(out)))
    return from_mont(out.reshape(12, 4), P_MOD)


def g2_mul(Q, k: int):
    g2 = np.zeros(16, dtype=np.uint64)
    g2[:] = to_mont([Q[0][0], Q[0][1], Q[1][0], Q[1][1]], P_MOD).reshape(-1)
    kk = np.array([(k % R_MOD >> (64 * i)) & ((1 << 64) - 1) for i in range(4)], dtype=np.uint64)
    out = np.zeros(16, dtype=np.uint64)
    _check(N.load().tns_g2_mul(N.p64(g2), N.p64(kk), N.p64(out)))
    if not out.any():
        return None
    v = from_mont(out.reshape(4, 4), P_MOD)
    return ((v[0], v[1]), (v[2], v[3]))


def profile_enable(ctx: Context, on: bool = True):
    N.load().tns_profile_enable(ctx.handle, 1 if on else 0)


def profile_only(ctx: Context, stage=None):
    """Time only `stage` (None: every stage) while profiling is enabled."""
    _check(N.load().tns_profile_only(ctx.handle, stage.encode() if stage else None))


PROFILE_STAGES = ["msm_digits", "msm_sort", "msm_accumulate", "msm_fixup", "msm_reduce", "ntt_stage", "ntt_lds",
                  "ntt_pointwise", "interp_tile", "interp_elementwise", "sumcheck_round", "open_scan"]


def profile_read_ex(ctx: Context, stage: str) -> dict:
    """Stage totals since profile_enable: summed launch ms, launches, algorithmic bytes,
    operations (msm_accumulate: mixed additions) and busy ms (union of launch intervals)."""
    out = (C.c_double * 5)()
    _check(N.load().tns_profile_read_ex(ctx.handle, stage.encode(), out))
    return dict(ms=out[0], launches=int(out[1]), bytes=out[2], ops=out[3], busy_ms=out[4])


def profile_read(ctx: Context, stage: str):
    """(device ms, launches, algorithmic bytes) accumulated for one stage since profile_enable."""
    ms = C.c_double()
    n = C.c_uint64()
    b = C.c_double()
    _check(N.load().tns_profile_read(ctx.handle, stage.encode(), C.byref(ms), C.byref(n), C.byref(b)))
    return ms.value, n.value, b.value


def fr_rand_batch(seed: bytes, n: int) -> np.ndarray:
    """n Fr::rand draws from ChaCha20Rng::from_seed(seed), Montgomery limbs."""
    out = np.empty((n, 4), dtype=np.uint64)
    if n:
        N.load().tns_fr_rand_batch((C.c_uint8 * 32)(*seed), n, N.p64(out))
    return out


def bench_trace(memory_size: int, n_ops: int):
    """Synthetic trace of src/benchmarks.rs:88-99 as SoA arrays (addr, value Montgomery, is_write)."""
    addr = np.empty(n_ops, dtype=np.uint64)
    val = np.empty(n_ops, dtype=np.uint64)
    isw = np.empty(n_ops, dtype=np.uint8)
    if n_ops:
        _check(N.load().tns_bench_trace(memory_size, n_ops, N.p64(addr), N.p64(val), N.p8(isw)))
    return addr, fr_from_u64_array(val), isw


__all__ = [
    "R_MOD", "P_MOD", "FieldElement", "TwistAndShoutError", "InvalidParameters", "ProofGeneration",
    "ProofVerification", "CommitmentError", "PolynomialError", "SumCheckError", "DeviceError", "Context",
    "CommitmentParams", "ProverParams", "VerifierParams", "setup_params", "Transcript", "KZGCommitment",
    "KZGCommitmentValue", "KZGProof", "msm", "poly_utils", "MultilinearExtension", "SumCheck", "SumCheckProof",
    "MemoryOp", "MemoryTrace", "Twist", "TwistProof", "LookupOp", "LookupTable", "Shout", "ShoutProof",
    "bench_trace", "to_mont", "from_mont", "fr_from_u64_array", "device_count", "Comm", "setup_params_shard",
    "shard_slice", "bench_trace_slice", "KZGVectorCommitment", "CommitmentVerificationKey", "pairing",
    "g1_serialize", "g1_deserialize",
]
