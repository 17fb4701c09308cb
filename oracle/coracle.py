"""ctypes binding of oracle/liboracle.so (the C restatement).  TEST INFRASTRUCTURE ONLY.

Converts between Python ints (canonical field values) and the arkworks memory
layout (uint64[4] Montgomery).  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module.
"""

from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from . import pyoracle as po

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

U64P = C.POINTER(C.c_uint64)
MAX_ROUNDS = 40


class OrcProof(C.Structure):
    _fields_ = [
        ("commitment", (C.c_uint64 * 8) * 2),
        ("num_rounds", C.c_uint32),
        ("num_openings", C.c_uint32),
        ("round_polynomials", ((C.c_uint64 * 4) * 4) * MAX_ROUNDS),
        ("final_evaluation", C.c_uint64 * 4),
        ("opening_proofs", (C.c_uint64 * 8) * 2),
        ("final_evaluations", (C.c_uint64 * 4) * 2),
        ("opening_point", C.c_uint64 * 4),
        ("sumcheck_challenges", (C.c_uint64 * 4) * MAX_ROUNDS),
    ]


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle.so"])


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.orc_setup_num_powers.restype = C.c_size_t
        L.orc_siphash.restype = C.c_uint64
        L.orc_siphash.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64, C.c_uint64, C.c_int, C.c_int]
        L.orc_chacha20_block.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p]
        _LIB = L
    return _LIB


# ----------------------------------------------------------------- conversions
def fr_array(vals, mod=po.R_MOD) -> np.ndarray:
    """ints -> (n,4) uint64 Montgomery array."""
    out = np.zeros((len(vals), 4), dtype=np.uint64)
    for i, v in enumerate(vals):
        out[i] = po.to_mont_limbs(int(v), mod)
    return out


def fr_ints(arr, mod=po.R_MOD):
    arr = np.asarray(arr, dtype=np.uint64).reshape(-1, 4)
    return [po.from_mont_limbs([int(x) for x in row], mod) for row in arr]


def g1_from_limbs(a):
    a = [int(x) for x in np.asarray(a, dtype=np.uint64).reshape(-1)]
    if not any(a[:8]):
        return None
    return (po.from_mont_limbs(a[0:4], po.P_MOD), po.from_mont_limbs(a[4:8], po.P_MOD))


def g1_to_limbs(P) -> np.ndarray:
    if P is None:
        return np.zeros(8, dtype=np.uint64)
    return np.concatenate([fr_array([P[0]], po.P_MOD)[0], fr_array([P[1]], po.P_MOD)[0]])


def _p(a: np.ndarray):
    return a.ctypes.data_as(U64P)


# ----------------------------------------------------------------- wrappers
def setup_params(log_size: int, with_srs: bool = True):
    L = lib()
    n = L.orc_setup_num_powers(C.c_uint(log_size))
    tau = np.zeros(4, dtype=np.uint64)
    seed = (C.c_uint8 * 32)()
    g1 = np.zeros((n, 8), dtype=np.uint64) if with_srs else None
    L.orc_setup_params(C.c_uint(log_size), _p(tau), seed, _p(g1) if with_srs else None)
    return dict(log_size=log_size, max_operations=1 << (log_size + 2), n_powers=n,
                tau_limbs=tau, tau=fr_ints(tau)[0], fiat_shamir_seed=bytes(seed), g1_limbs=g1)


def interpolate(y_limbs: np.ndarray) -> np.ndarray:
    y = np.ascontiguousarray(y_limbs, dtype=np.uint64).reshape(-1, 4)
    out = np.zeros_like(y)
    lib().orc_interpolate_consecutive(_p(y), C.c_size_t(len(y)), _p(out))
    return out


def commit(g1_limbs, coeff_limbs):
    c = np.ascontiguousarray(coeff_limbs, dtype=np.uint64).reshape(-1, 4)
    g = np.ascontiguousarray(g1_limbs, dtype=np.uint64)
    out = np.zeros(8, dtype=np.uint64)
    st = lib().orc_commit(_p(g), C.c_size_t(len(g)), _p(c), C.c_size_t(len(c)), _p(out))
    return st, out


def open_(g1_limbs, coeff_limbs, z_limbs):
    c = np.ascontiguousarray(coeff_limbs, dtype=np.uint64).reshape(-1, 4)
    g = np.ascontiguousarray(g1_limbs, dtype=np.uint64)
    z = np.ascontiguousarray(z_limbs, dtype=np.uint64).reshape(4)
    v = np.zeros(4, dtype=np.uint64)
    pi = np.zeros(8, dtype=np.uint64)
    st = lib().orc_open(_p(g), C.c_size_t(len(g)), _p(c), C.c_size_t(len(c)), _p(z), _p(v), _p(pi))
    return st, v, pi


def mle_evaluate(evals, point):
    e = np.ascontiguousarray(evals, dtype=np.uint64).reshape(-1, 4)
    p = np.ascontiguousarray(point, dtype=np.uint64).reshape(-1, 4)
    out = np.zeros(4, dtype=np.uint64)
    lib().orc_mle_evaluate(_p(e), C.c_uint(len(p)), _p(p), _p(out))
    return out


def mle_partial_evaluate(evals, fixed):
    e = np.ascontiguousarray(evals, dtype=np.uint64).reshape(-1, 4)
    f = np.ascontiguousarray(fixed, dtype=np.uint64).reshape(-1, 4)
    nv = len(e).bit_length() - 1
    out = np.zeros((1 << (nv - len(f)), 4), dtype=np.uint64)
    lib().orc_mle_partial_evaluate(_p(e), C.c_uint(nv), _p(f), C.c_uint(len(f)), _p(out))
    return out


def sumcheck_prove(tables, nv, claimed, terms, prefix: bytes = b""):
    """terms: list of (coeff_int, [table indices]) with <= 3 factors each."""
    arrs = [np.ascontiguousarray(t, dtype=np.uint64).reshape(-1, 4) for t in tables]
    ptrs = (U64P * max(1, len(arrs)))(*[_p(a) for a in arrs])
    coeffs = fr_array([c for c, _ in terms]) if terms else np.zeros((1, 4), dtype=np.uint64)
    tt = np.full((max(1, len(terms)), 3), -1, dtype=np.int32)
    for i, (_, ix) in enumerate(terms):
        tt[i, : len(ix)] = ix
    cl = fr_array([claimed])[0]
    rounds = np.zeros((max(1, nv), 4, 4), dtype=np.uint64)
    fin = np.zeros(4, dtype=np.uint64)
    chal = np.zeros((max(1, nv), 4), dtype=np.uint64)
    pre = (C.c_uint8 * max(1, len(prefix))).from_buffer_copy(prefix or b"\0")
    st = lib().orc_sumcheck_prove(ptrs, C.c_int(len(arrs)), C.c_uint(nv), _p(cl), C.c_int(len(terms)),
                                  _p(coeffs), tt.ctypes.data_as(C.POINTER(C.c_int)), pre,
                                  C.c_size_t(len(prefix)), _p(rounds), _p(fin), _p(chal))
    return st, rounds[:nv], fin, chal[:nv]


def _terms_arrays(terms):
    coeffs = fr_array([c for c, _ in terms]) if terms else np.zeros((1, 4), dtype=np.uint64)
    tt = np.full((max(1, len(terms)), 3), -1, dtype=np.int32)
    for i, (_, ix) in enumerate(terms):
        tt[i, : len(ix)] = ix
    return coeffs, tt


def fast_sumcheck_prove(tables, nv, claimed, terms, prefix: bytes = b"", threads=1):
    """fastcpu.c fc_sumcheck_prove: the same outputs as sumcheck_prove with O(N)-per-round folds
    on `threads` host threads.  tables: (2^nv, 4) Montgomery arrays; claimed: int or None (the
    honest sum, fast_composition_sum)."""
    arrs = [np.ascontiguousarray(t, dtype=np.uint64).reshape(-1, 4) for t in tables]
    ptrs = (U64P * max(1, len(arrs)))(*[_p(a) for a in arrs])
    coeffs, tt = _terms_arrays(terms)
    if claimed is None:
        claimed = fast_composition_sum(arrs, nv, terms, threads)
    cl = fr_array([claimed])[0]
    rounds = np.zeros((max(1, nv), 4, 4), dtype=np.uint64)
    fin = np.zeros(4, dtype=np.uint64)
    chal = np.zeros((max(1, nv), 4), dtype=np.uint64)
    pre = (C.c_uint8 * max(1, len(prefix))).from_buffer_copy(prefix or b"\0")
    st = lib().fc_sumcheck_prove(ptrs, C.c_int(len(arrs)), C.c_uint(nv), _p(cl), C.c_int(len(terms)), _p(coeffs),
                                 tt.ctypes.data_as(C.POINTER(C.c_int)), pre, C.c_size_t(len(prefix)),
                                 C.c_int(threads), _p(rounds), _p(fin), _p(chal))
    return st, rounds[:nv], fin, chal[:nv]


def fast_composition_sum(tables, nv, terms, threads=1) -> int:
    arrs = [np.ascontiguousarray(t, dtype=np.uint64).reshape(-1, 4) for t in tables]
    ptrs = (U64P * max(1, len(arrs)))(*[_p(a) for a in arrs])
    coeffs, tt = _terms_arrays(terms)
    out = np.zeros(4, dtype=np.uint64)
    lib().fc_composition_sum(ptrs, C.c_uint(nv), C.c_int(len(terms)), _p(coeffs),
                             tt.ctypes.data_as(C.POINTER(C.c_int)), C.c_int(threads), _p(out))
    return fr_ints(out)[0]


def _proof_dict(pr: OrcProof, names):
    nr = pr.num_rounds
    rounds = np.ctypeslib.as_array(pr.round_polynomials)[:nr]
    return {
        names[0]: g1_from_limbs(np.ctypeslib.as_array(pr.commitment[0])),
        names[1]: g1_from_limbs(np.ctypeslib.as_array(pr.commitment[1])),
        "round_polynomials": [fr_ints(r) for r in rounds],
        "final_evaluation": fr_ints(np.ctypeslib.as_array(pr.final_evaluation))[0],
        "opening_proofs": [g1_from_limbs(np.ctypeslib.as_array(pr.opening_proofs[i]))
                           for i in range(pr.num_openings)],
        "final_evaluations": [fr_ints(np.ctypeslib.as_array(pr.final_evaluations[i]))[0]
                              for i in range(pr.num_openings)],
        "opening_point": (fr_ints(np.ctypeslib.as_array(pr.opening_point))[0]
                          if pr.num_openings else None),
        "sumcheck_challenges": fr_ints(np.ctypeslib.as_array(pr.sumcheck_challenges)[:nr]) if nr else [],
    }


def twist_prove(params, ops):
    """ops: list of (is_write, addr, value_int)."""
    g = params["g1_limbs"]
    n = len(ops)
    addr = fr_array([a for (_, a, _) in ops]) if n else np.zeros((1, 4), dtype=np.uint64)
    val = fr_array([v for (_, _, v) in ops]) if n else np.zeros((1, 4), dtype=np.uint64)
    isw = np.array([w for (w, _, _) in ops] or [0], dtype=np.uint8)
    pr = OrcProof()
    st = lib().orc_twist_prove(_p(g), C.c_size_t(len(g)), C.c_size_t(params["max_operations"]),
                               _p(addr), _p(val), isw.ctypes.data_as(C.POINTER(C.c_uint8)),
                               C.c_size_t(n), C.byref(pr))
    return st, _proof_dict(pr, ("address_commitment", "value_commitment"))


def shout_prove(params, entries, indices):
    g = params["g1_limbs"]
    e = fr_array(entries) if entries else np.zeros((1, 4), dtype=np.uint64)
    ix = fr_array(indices) if indices else np.zeros((1, 4), dtype=np.uint64)
    pr = OrcProof()
    st = lib().orc_shout_prove(_p(g), C.c_size_t(len(g)), C.c_size_t(params["max_operations"]),
                               _p(e), C.c_size_t(len(entries)), _p(ix), C.c_size_t(len(indices)),
                               C.byref(pr))
    return st, _proof_dict(pr, ("table_commitment", "index_commitment"))


def horner(coeff_limbs, z_limbs):
    c = np.ascontiguousarray(coeff_limbs, dtype=np.uint64).reshape(-1, 4)
    z = np.ascontiguousarray(z_limbs, dtype=np.uint64).reshape(4)
    out = np.zeros(4, dtype=np.uint64)
    lib().orc_horner(_p(c), C.c_size_t(len(c)), _p(z), _p(out))
    return out


# ----------------------------------------------------------------- fast CPU baseline (fastcpu.c)
def bary_weights(N: int) -> np.ndarray:
    w = np.zeros((N, 4), dtype=np.uint64)
    lib().fc_bary_weights(C.c_size_t(N), _p(w))
    return w


def lagrange_basis(tau_limbs, N: int) -> np.ndarray:
    """[L_j(tau)]G for the nodes 0..N-1 (affine limbs), by scalar multiplication: small N."""
    t = np.ascontiguousarray(tau_limbs, dtype=np.uint64).reshape(4)
    out = np.zeros((N, 8), dtype=np.uint64)
    lib().fc_lagrange_basis(_p(t), C.c_size_t(N), _p(out))
    return out


def fast_twist_prove(lagrange, bary_w, max_ops, addr_u64, val_limbs, is_write, threads=1):
    """Twist::prove with the GPU path's algorithms on `threads` host threads (fastcpu.c).
    addr_u64: uint64 addresses, val_limbs: (n,4) Montgomery Fr, is_write: uint8."""
    lag = np.ascontiguousarray(lagrange, dtype=np.uint64).reshape(-1, 8)
    w = np.ascontiguousarray(bary_w, dtype=np.uint64).reshape(-1, 4)
    a = np.ascontiguousarray(addr_u64, dtype=np.uint64)
    v = np.ascontiguousarray(val_limbs, dtype=np.uint64).reshape(-1, 4)
    isw = np.ascontiguousarray(is_write, dtype=np.uint8)
    pr = OrcProof()
    st = lib().fc_twist_prove(_p(lag), _p(w), C.c_size_t(len(lag)), C.c_size_t(max_ops), _p(a), _p(v),
                              isw.ctypes.data_as(C.POINTER(C.c_uint8)), C.c_size_t(len(a)), C.c_int(threads),
                              C.byref(pr))
    return st, _proof_dict(pr, ("address_commitment", "value_commitment"))


def bary_eval2(bary_w, y0_limbs, y1_limbs, x: int, threads=1):
    """(f0(x), f1(x), ell(x)) as ints for two vectors of N evaluations on the nodes 0..N-1
    (Montgomery limbs; y1 may be y0): the barycentric formula in O(N) on `threads` host threads
    (fastcpu.c fc_bary_eval2).  Size-independent parity checks of commitments and openings
    (C = f(tau) G, pi (tau - z) = C - v G).  x must not be a node."""
    w = np.ascontiguousarray(bary_w, dtype=np.uint64).reshape(-1, 4)
    y0 = np.ascontiguousarray(y0_limbs, dtype=np.uint64).reshape(-1, 4)
    y1 = np.ascontiguousarray(y1_limbs, dtype=np.uint64).reshape(-1, 4)
    assert len(w) == len(y0) == len(y1)
    xl = fr_array([x])[0]
    f0, f1, ell = (np.zeros(4, dtype=np.uint64) for _ in range(3))
    st = lib().fc_bary_eval2(_p(w), _p(y0), _p(y1), C.c_size_t(len(w)), _p(xl), C.c_int(threads), _p(f0), _p(f1),
                             _p(ell))
    assert st == 0, "x is an interpolation node"
    return fr_ints(f0)[0], fr_ints(f1)[0], fr_ints(ell)[0]


def g1_mul_gen(k: int):
    """k * G1 (affine ints, None = identity), by the C oracle's double-and-add."""
    out = np.zeros(8, dtype=np.uint64)
    lib().fc_g1_mul_gen(_p(fr_array([k % po.R_MOD])[0]), _p(out))
    return g1_from_limbs(out)


def g1_mul(P, k: int):
    """k * P for an affine point P (ints, None = identity)."""
    out = np.zeros(8, dtype=np.uint64)
    lib().fc_g1_mul(_p(g1_to_limbs(P)), _p(fr_array([k % po.R_MOD])[0]), _p(out))
    return g1_from_limbs(out)
