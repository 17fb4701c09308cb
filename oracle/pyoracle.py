"""Pure-Python CPU restatement of the twist-and-shout prover (TEST INFRASTRUCTURE ONLY).

This file is the *oracle*: a slow, line-by-line restatement of the reference
crate's prover semantics, used only by ``tests/``, ``tests/golden/gen_golden.py``
and ``__graft_entry__.smoke()`` as a checker.  Nothing in the product path
(``multilinear-map-cryptography_amd/``) may import it.

Reference: /root/reference (crate ``twist-and-shout``, Rust, arkworks 0.4).
Every function cites the reference file:line it restates.  Arithmetic that
lives in un-vendored third-party crates is restated from their published
algorithms (pinned versions from ``Cargo.lock``):

* ark-ff 0.4.2 / ark-bn254 0.4.0 -- BN254 Fr/Fq (Montgomery, R = 2^256),
  ``UniformRand for Fp`` (4 x next_u64, mask top 2 bits, reject >= modulus,
  limbs taken *as the Montgomery representation*), ``from_le_bytes_mod_order``,
  compressed serialisation of Fr = 32-byte little-endian canonical integer.
* ark-ec 0.4.2 -- short-Weierstrass Jacobian G1 (y^2 = x^3 + 3, generator (1,2)),
  ``into_affine`` of the identity has x = 0.
* rand_chacha 0.3.1 / rand_core 0.6.4 -- ``ChaCha20Rng::from_seed``: DJB ChaCha20,
  key = seed, 64-bit block counter from 0, stream 0; output consumed as a stream
  of little-endian u32 words; ``next_u64 = w[i] | w[i+1] << 32``.
* Rust std 1.89 ``DefaultHasher`` = SipHash-1-3 with keys (0, 0);
  ``Hash for Vec<u8>`` = ``write_usize(len)`` (8 LE bytes) followed by the bytes.

Parity status (see DESIGN.md "Oracle"): the reference's own known-answer tests
(tests/polynomial_tests.rs, src/commitments.rs tests, src/utils.rs tests) and the
published ChaCha20 / SipHash-2-4 test vectors pin this restatement; transcript
bytes, tau, SRS points and whole proofs are *parity unpinned* against a run of
the real Rust binary (no Rust toolchain exists in this environment).
"""

from __future__ import annotations

import struct

# ----------------------------------------------------------------------------
# Field constants (ark-bn254 0.4.0)
# ----------------------------------------------------------------------------
R_MOD = 0x30644E72E131A029B85045B68181585D2833E84879B9709143E1F593F0000001  # Fr
P_MOD = 0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47  # Fq
MONT_R = 1 << 256
MASK64 = (1 << 64) - 1
MASK32 = (1 << 32) - 1
G1_B = 3
G1_GEN = (1, 2)


def fr(x: int) -> int:
    return x % R_MOD


def fr_inv(x: int) -> int:
    if x % R_MOD == 0:
        raise ZeroDivisionError("Fr inverse of zero")
    return pow(x, R_MOD - 2, R_MOD)


def to_mont_limbs(x: int, mod: int = R_MOD) -> list[int]:
    """Canonical value -> arkworks memory layout (4 x u64 LE, Montgomery form)."""
    m = (x % mod) * MONT_R % mod
    return [(m >> (64 * i)) & MASK64 for i in range(4)]


def from_mont_limbs(limbs, mod: int = R_MOD) -> int:
    m = sum(int(l) << (64 * i) for i, l in enumerate(limbs))
    return m * pow(MONT_R, -1, mod) % mod


def fr_to_bytes_le(x: int) -> bytes:
    """ark-serialize compressed Fr: 32-byte LE canonical (src/utils.rs:155-158)."""
    return (x % R_MOD).to_bytes(32, "little")


# ----------------------------------------------------------------------------
# ChaCha20Rng (rand_chacha 0.3.1), restated
# ----------------------------------------------------------------------------
def _rotl32(v, c):
    return ((v << c) & MASK32) | (v >> (32 - c))


def chacha20_block(key_words, counter: int, stream: int = 0) -> list[int]:
    """DJB ChaCha20 block function: 64-bit counter in words 12-13, stream in 14-15."""
    st = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574] + list(key_words) + [
        counter & MASK32, (counter >> 32) & MASK32, stream & MASK32, (stream >> 32) & MASK32]
    x = list(st)

    def qr(a, b, c, d):
        x[a] = (x[a] + x[b]) & MASK32; x[d] = _rotl32(x[d] ^ x[a], 16)
        x[c] = (x[c] + x[d]) & MASK32; x[b] = _rotl32(x[b] ^ x[c], 12)
        x[a] = (x[a] + x[b]) & MASK32; x[d] = _rotl32(x[d] ^ x[a], 8)
        x[c] = (x[c] + x[d]) & MASK32; x[b] = _rotl32(x[b] ^ x[c], 7)

    for _ in range(10):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    return [(x[i] + st[i]) & MASK32 for i in range(16)]


def chacha20_block_raw(state16) -> list[int]:
    """Block function on an arbitrary 16-word input state (for RFC 8439 vectors)."""
    x = list(state16)
    st = list(state16)

    def qr(a, b, c, d):
        x[a] = (x[a] + x[b]) & MASK32; x[d] = _rotl32(x[d] ^ x[a], 16)
        x[c] = (x[c] + x[d]) & MASK32; x[b] = _rotl32(x[b] ^ x[c], 12)
        x[a] = (x[a] + x[b]) & MASK32; x[d] = _rotl32(x[d] ^ x[a], 8)
        x[c] = (x[c] + x[d]) & MASK32; x[b] = _rotl32(x[b] ^ x[c], 7)

    for _ in range(10):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    return [(x[i] + st[i]) & MASK32 for i in range(16)]


class ChaCha20Rng:
    """``ChaCha20Rng::from_seed`` + rand_core ``BlockRng`` word stream."""

    def __init__(self, seed: bytes):
        assert len(seed) == 32
        self.key = list(struct.unpack("<8I", seed))
        self.counter = 0
        self.buf: list[int] = []
        self.idx = 0

    def _refill(self):
        # rand_chacha buffers 4 blocks (64 words); word order is sequential.
        self.buf = []
        for _ in range(4):
            self.buf += chacha20_block(self.key, self.counter)
            self.counter += 1
        self.idx = 0

    def next_u32(self) -> int:
        if self.idx >= len(self.buf):
            self._refill()
        v = self.buf[self.idx]
        self.idx += 1
        return v

    def next_u64(self) -> int:
        # BlockRng::next_u64: low word first; straddling a refill takes the
        # last word of the old buffer as the low half (rand_core 0.6.4).
        lo = self.next_u32()
        hi = self.next_u32()
        return lo | (hi << 32)

    def fill_bytes(self, n: int) -> bytes:
        out = b""
        while len(out) < n:
            out += struct.pack("<I", self.next_u32())
        return out[:n]


def fr_rand(rng: ChaCha20Rng) -> int:
    """ark-ff 0.4.2 ``UniformRand for Fp<P,4>`` on BN254 Fr (254-bit: shave 2 bits).

    The sampled limbs ARE the Montgomery representation, so the canonical value
    is limbs * R^-1 mod r.
    """
    while True:
        limbs = [rng.next_u64() for _ in range(4)]
        limbs[3] &= MASK64 >> 2
        v = sum(l << (64 * i) for i, l in enumerate(limbs))
        if v < R_MOD:
            return v * pow(MONT_R, -1, R_MOD) % R_MOD


# ----------------------------------------------------------------------------
# SipHash (Rust std DefaultHasher = SipHash-1-3, keys 0,0)
# ----------------------------------------------------------------------------
def _rotl64(v, c):
    return ((v << c) & MASK64) | (v >> (64 - c))


def siphash(msg: bytes, k0: int = 0, k1: int = 0, c_rounds: int = 1, d_rounds: int = 3) -> int:
    v0 = k0 ^ 0x736F6D6570736575
    v1 = k1 ^ 0x646F72616E646F6D
    v2 = k0 ^ 0x6C7967656E657261
    v3 = k1 ^ 0x7465646279746573

    def rnd():
        nonlocal v0, v1, v2, v3
        v0 = (v0 + v1) & MASK64; v1 = _rotl64(v1, 13); v1 ^= v0; v0 = _rotl64(v0, 32)
        v2 = (v2 + v3) & MASK64; v3 = _rotl64(v3, 16); v3 ^= v2
        v0 = (v0 + v3) & MASK64; v3 = _rotl64(v3, 21); v3 ^= v0
        v2 = (v2 + v1) & MASK64; v1 = _rotl64(v1, 17); v1 ^= v2; v2 = _rotl64(v2, 32)

    n = len(msg)
    full = n - n % 8
    for off in range(0, full, 8):
        m = struct.unpack_from("<Q", msg, off)[0]
        v3 ^= m
        for _ in range(c_rounds):
            rnd()
        v0 ^= m
    tail = 0
    for i, b in enumerate(msg[full:]):
        tail |= b << (8 * i)
    b = ((n & 0xFF) << 56) | tail
    v3 ^= b
    for _ in range(c_rounds):
        rnd()
    v0 ^= b
    v2 ^= 0xFF
    for _ in range(d_rounds):
        rnd()
    return v0 ^ v1 ^ v2 ^ v3


def rust_default_hash_bytes(state: bytes) -> int:
    """``Vec<u8>::hash`` into ``DefaultHasher``: write_usize(len) then the bytes."""
    return siphash(struct.pack("<Q", len(state)) + state, 0, 0, 1, 3)


# ----------------------------------------------------------------------------
# Transcript (src/utils.rs:134-204)
# ----------------------------------------------------------------------------
class Transcript:
    def __init__(self, seed: bytes):
        # src/utils.rs:141-147 -- the seeded rng is overwritten before any use.
        self.state = bytearray()

    def append_field_element(self, label: bytes, x: int):  # src/utils.rs:150-159
        self.state += label
        self.state += fr_to_bytes_le(x)

    def append_field_elements(self, label: bytes, xs):  # src/utils.rs:162-169
        self.state += label
        for x in xs:
            self.state += fr_to_bytes_le(x)

    def challenge_field_element(self, label: bytes) -> int:  # src/utils.rs:172-192
        self.state += label
        h = rust_default_hash_bytes(bytes(self.state))
        seed = struct.pack("<Q", h) * 4
        return fr_rand(ChaCha20Rng(seed))

    def challenge_field_elements(self, label: bytes, count: int):  # src/utils.rs:195-203
        return [self.challenge_field_element(label + b"_" + str(i).encode()) for i in range(count)]


# ----------------------------------------------------------------------------
# BN254 G1 (ark-bn254 0.4.0), Jacobian
# ----------------------------------------------------------------------------
INF = None  # affine identity


def g1_is_on_curve(P) -> bool:
    if P is None:
        return True
    x, y = P
    return (y * y - x * x * x - G1_B) % P_MOD == 0


def jac_double(P):
    X, Y, Z = P
    if Z == 0 or Y == 0:
        return (1, 1, 0)
    p = P_MOD
    A = X * X % p
    B = Y * Y % p
    C = B * B % p
    D = 2 * ((X + B) * (X + B) - A - C) % p
    E = 3 * A % p
    F = E * E % p
    X3 = (F - 2 * D) % p
    Y3 = (E * (D - X3) - 8 * C) % p
    Z3 = 2 * Y * Z % p
    return (X3, Y3, Z3)


def jac_add(P, Q):
    if P[2] == 0:
        return Q
    if Q[2] == 0:
        return P
    p = P_MOD
    X1, Y1, Z1 = P
    X2, Y2, Z2 = Q
    Z1Z1 = Z1 * Z1 % p
    Z2Z2 = Z2 * Z2 % p
    U1 = X1 * Z2Z2 % p
    U2 = X2 * Z1Z1 % p
    S1 = Y1 * Z2 * Z2Z2 % p
    S2 = Y2 * Z1 * Z1Z1 % p
    if U1 == U2:
        if S1 == S2:
            return jac_double(P)
        return (1, 1, 0)
    H = (U2 - U1) % p
    I = (2 * H) * (2 * H) % p
    J = H * I % p
    rr = 2 * (S2 - S1) % p
    V = U1 * I % p
    X3 = (rr * rr - J - 2 * V) % p
    Y3 = (rr * (V - X3) - 2 * S1 * J) % p
    Z3 = ((Z1 + Z2) * (Z1 + Z2) - Z1Z1 - Z2Z2) * H % p
    return (X3, Y3, Z3)


def to_jac(A):
    if A is None:
        return (1, 1, 0)
    return (A[0], A[1], 1)


def to_affine(P):
    X, Y, Z = P
    if Z == 0:
        return None
    zi = pow(Z, P_MOD - 2, P_MOD)
    zi2 = zi * zi % P_MOD
    return (X * zi2 % P_MOD, Y * zi2 * zi % P_MOD)


def g1_neg(A):
    if A is None:
        return None
    return (A[0], (-A[1]) % P_MOD)


def jac_mul(P, k: int):
    """Double-and-add scalar multiplication (``G1Projective * Fr``)."""
    k %= R_MOD
    acc = (1, 1, 0)
    for bit in bin(k)[2:] if k else "":
        acc = jac_double(acc)
        if bit == "1":
            acc = jac_add(acc, P)
    return acc


def affine_mul(A, k: int):
    return to_affine(jac_mul(to_jac(A), k))


def affine_add(A, B):
    return to_affine(jac_add(to_jac(A), to_jac(B)))


# ----------------------------------------------------------------------------
# setup_params (src/utils.rs:79-131)
# ----------------------------------------------------------------------------
def next_pow2(n: int) -> int:
    """Rust ``usize::next_power_of_two`` (0 -> 1)."""
    if n <= 1:
        return 1
    return 1 << (n - 1).bit_length()


def setup_params(log_size: int, with_srs: bool = True):
    """Returns dict(log_size, max_operations, tau, g1_powers (affine list), fiat_shamir_seed)."""
    max_operations = 1 << (log_size + 2)  # src/utils.rs:80
    rng = ChaCha20Rng(bytes([42] * 32))  # :81
    tau = fr_rand(rng)  # :84
    max_degree = next_pow2(max_operations)  # :89
    g1 = None
    if with_srs:
        g1 = []
        cur = 1
        for _ in range(max_degree + 1):  # :93-96
            g1.append(affine_mul(G1_GEN, cur))
            cur = cur * tau % R_MOD
    seed = rng.fill_bytes(32)  # :101-102
    return dict(log_size=log_size, max_operations=max_operations, tau=tau,
                n_powers=max_degree + 1, g1_powers=g1, fiat_shamir_seed=seed)


# ----------------------------------------------------------------------------
# Polynomials (src/polynomials.rs)
# ----------------------------------------------------------------------------
def lagrange_interpolate(points):
    """src/polynomials.rs:301-352, verbatim O(n^3) algorithm."""
    n = len(points)
    if n == 0:
        return []
    result = [0] * n
    for i in range(n):
        xi, yi = points[i]
        li = [1]
        for j in range(n):
            if i == j:
                continue
            xj = points[j][0]
            dinv = fr_inv(xi - xj)
            new = [0] * (len(li) + 1)
            for k in range(len(li)):
                new[k + 1] = (new[k + 1] + li[k]) % R_MOD
            for k in range(len(li)):
                new[k] = (new[k] - li[k] * xj) % R_MOD
            li = [c * dinv % R_MOD for c in new]
        for k in range(min(len(li), n)):
            result[k] = (result[k] + yi * li[k]) % R_MOD
    return result


def vector_to_polynomial(vec):
    """src/twist.rs:307-315 / src/shout.rs:277-285: interpolate over {0..n-1}."""
    return lagrange_interpolate([(i, v % R_MOD) for i, v in enumerate(vec)])


def horner_eval(coeffs, z: int) -> int:
    """src/utils.rs:217-221 and src/commitments.rs:305-313."""
    acc = 0
    for c in reversed(coeffs):
        acc = (acc * z + c) % R_MOD
    return acc


def polynomial_division(dividend, divisor):
    """src/commitments.rs:338-375 (quotient only)."""
    if not divisor or all(d % R_MOD == 0 for d in divisor):
        raise ValueError("Polynomial: Cannot divide by zero polynomial")
    rem = [c % R_MOD for c in dividend]
    dd = len(divisor) - 1
    lead = divisor[dd] % R_MOD
    if lead == 0:
        raise ValueError("Polynomial: Divisor must have non-zero leading coefficient")
    linv = fr_inv(lead)
    if len(rem) < len(divisor):
        return []
    qd = len(rem) - len(divisor)
    q = [0] * (qd + 1)
    for i in range(qd, -1, -1):
        if len(rem) > i + dd:
            c = rem[i + dd] * linv % R_MOD
            q[i] = c
            for j in range(len(divisor)):
                if i + j < len(rem):
                    rem[i + j] = (rem[i + j] - c * divisor[j]) % R_MOD
    return q


def compute_quotient_polynomial(poly, z, v):
    """src/commitments.rs:317-334."""
    if not poly:
        return []
    shifted = list(poly)
    shifted[0] = (shifted[0] - v) % R_MOD
    return polynomial_division(shifted, [(-z) % R_MOD, 1])


class CommitmentError(Exception):
    pass


def kzg_commit(g1_powers, poly):
    """src/commitments.rs:162-180 (sequential per-term scalar mult + sum)."""
    if len(poly) > len(g1_powers):
        raise CommitmentError("Polynomial degree exceeds setup size")
    acc = (1, 1, 0)
    for c, g in zip(poly, g1_powers):
        acc = jac_add(acc, jac_mul(to_jac(g), c))
    return to_affine(acc)


def kzg_open(g1_powers, poly, z):
    """src/commitments.rs:182-199: (value, proof)."""
    v = horner_eval(poly, z) if poly else 0
    q = compute_quotient_polynomial(poly, z, v)
    return v, kzg_commit(g1_powers, q)


def commitment_hash(C) -> int:
    """src/commitments.rs:73-84: affine x (canonical, LE bytes) reduced mod r."""
    if C is None:
        return 0
    return C[0] % R_MOD


# ----------------------------------------------------------------------------
# MultilinearExtension (src/polynomials.rs:18-196)
# ----------------------------------------------------------------------------
def mle_basis(index: int, point) -> int:  # src/polynomials.rs:108-122
    res = 1
    for j, rj in enumerate(point):
        res = res * (rj if (index >> j) & 1 else (1 - rj)) % R_MOD
    return res


def mle_evaluate(evals, point) -> int:  # src/polynomials.rs:85-103
    n = len(point)
    assert len(evals) == 1 << n, "Point dimension must match number of variables"
    acc = 0
    for i, e in enumerate(evals):
        if e % R_MOD == 0:
            continue
        acc = (acc + e * mle_basis(i, point)) % R_MOD
    return acc


def mle_partial_evaluate(evals, fixed):  # src/polynomials.rs:126-161
    n = (len(evals) - 1).bit_length() if len(evals) > 1 else 0
    k = len(fixed)
    assert k <= n
    if k == 0:
        return list(evals)
    nn = n - k
    out = []
    for idx in range(1 << nn):
        pt = list(fixed) + [(idx >> j) & 1 for j in range(nn)]
        out.append(mle_evaluate(evals, pt))
    return out


def mle_from_evaluations_vec(num_vars: int, evals):  # src/polynomials.rs:40-50
    size = 1 << num_vars
    e = list(evals[:size])
    return e + [0] * (size - len(e))


# ----------------------------------------------------------------------------
# SumCheck (src/sumcheck.rs:56-212)
# ----------------------------------------------------------------------------
class SumCheckError(Exception):
    pass


def sumcheck_prove(num_vars: int, claimed_sum: int, poly, transcript: Transcript):
    """Returns (round_polynomials, final_evaluation, challenges)."""
    rounds = []
    cur = claimed_sum % R_MOD
    fixed = []
    for rnd in range(num_vars):
        remaining = num_vars - len(fixed) - 1
        evs = []
        for xv in range(4):  # src/sumcheck.rs:175-198
            s = 0
            for suf in range(1 << remaining):
                pt = list(fixed) + [xv] + [(suf >> b) & 1 for b in range(remaining)]
                s = (s + poly(pt)) % R_MOD
            evs.append(s)
        coeffs = lagrange_interpolate([(i, evs[i]) for i in range(4)])  # :201-206
        g0 = horner_eval(coeffs, 0)
        g1 = horner_eval(coeffs, 1)
        if (g0 + g1) % R_MOD != cur:  # :80-84
            raise SumCheckError(f"Round {rnd} consistency check failed")
        rounds.append(coeffs)
        transcript.append_field_elements(f"sumcheck_round_{rnd}".encode(), coeffs)
        ch = transcript.challenge_field_element(f"sumcheck_challenge_{rnd}".encode())
        fixed.append(ch)
        cur = horner_eval(coeffs, ch)
    final = poly(fixed) % R_MOD
    return rounds, final, fixed


# ----------------------------------------------------------------------------
# Twist (src/twist.rs:107-252)
# ----------------------------------------------------------------------------
class InvalidParameters(Exception):
    pass


def memory_trace_ops(memory_size: int, script):
    """Replays MemoryTrace::write/read (src/twist.rs:37-71).

    ``script`` is a list of ("w", addr, value) / ("r", addr).  Returns a list of
    (is_write, addr, value) operations.
    """
    mem = [0] * memory_size
    ops = []
    for s in script:
        if s[0] == "w":
            _, a, v = s
            if a >= memory_size:
                raise InvalidParameters("Address out of bounds")
            mem[a] = v % R_MOD
            ops.append((1, a, v % R_MOD))
        else:
            a = s[1]
            if a >= memory_size:
                raise InvalidParameters("Address out of bounds")
            ops.append((0, a, mem[a]))
    return ops


def benchmark_trace(memory_size: int, num_ops: int):
    """src/benchmarks.rs:88-99 synthetic trace generator."""
    script = []
    for i in range(num_ops):
        if i % 3 == 0:
            script.append(("w", i % memory_size, i * 42))
        else:
            script.append(("r", (i // 2) % memory_size))
    return memory_trace_ops(memory_size, script)


def _log2_exact(n: int) -> int:
    return n.bit_length() - 1


def twist_prove(params, ops, keep_mle_evals: bool = True):
    """src/twist.rs:107-252.  ``ops`` = list of (is_write, addr, value)."""
    if len(ops) > params["max_operations"]:
        raise InvalidParameters("Too many operations")
    addrs = [a for (_, a, _) in ops]
    vals = [v for (_, _, v) in ops]
    opt = [w for (w, _, _) in ops]
    n_pad = max(next_pow2(len(addrs)), 1)
    addrs += [0] * (n_pad - len(addrs))
    vals += [0] * (n_pad - len(vals))
    opt += [0] * (n_pad - len(opt))
    a_poly = vector_to_polynomial(addrs)
    v_poly = vector_to_polynomial(vals)
    g1 = params["g1_powers"]
    C_a = kzg_commit(g1, a_poly)
    C_v = kzg_commit(g1, v_poly)
    log_ops = _log2_exact(n_pad)
    tr = Transcript(params["fiat_shamir_seed"])
    tr.append_field_element(b"address_commitment", commitment_hash(C_a))
    tr.append_field_element(b"value_commitment", commitment_hash(C_v))
    a_mle = mle_from_evaluations_vec(log_ops, addrs)
    v_mle = mle_from_evaluations_vec(log_ops, vals)
    o_mle = mle_from_evaluations_vec(log_ops, opt)
    mle_evals = []

    def consistency(vars_):  # src/twist.rs:191-213
        if len(vars_) != log_ops:
            return 0
        ca = mle_evaluate(a_mle, vars_)
        cv = mle_evaluate(v_mle, vars_)
        co = mle_evaluate(o_mle, vars_)
        if keep_mle_evals:
            mle_evals.append((ca, cv, co))
        return 0

    rounds, final, chals = sumcheck_prove(log_ops, 0, consistency, tr)
    opening = tr.challenge_field_elements(b"opening_challenges", log_ops)
    openings, finals = [], []
    if opening:
        z = opening[0]
        va, pa = kzg_open(g1, a_poly, z)
        vv, pv = kzg_open(g1, v_poly, z)
        openings = [pa, pv]
        finals = [va, vv]
    return dict(address_commitment=C_a, value_commitment=C_v,
                round_polynomials=rounds, final_evaluation=final,
                opening_proofs=openings, final_evaluations=finals,
                sumcheck_challenges=chals,
                opening_point=opening[0] if opening else None,
                final_mle_evals=(mle_evals[-1] if (mle_evals and log_ops) else None),
                address_poly=a_poly, value_poly=v_poly)


# ----------------------------------------------------------------------------
# Shout (src/shout.rs:97-222)
# ----------------------------------------------------------------------------
def shout_prove(params, entries, lookup_indices):
    if len(lookup_indices) > params["max_operations"]:
        raise InvalidParameters("Too many lookup operations")
    for i in lookup_indices:
        if i >= len(entries):
            raise InvalidParameters("Lookup index out of bounds")
    t_size = next_pow2(len(entries))
    table = [e % R_MOD for e in entries] + [0] * (t_size - len(entries))
    idx = list(lookup_indices)
    l_size = max(next_pow2(len(idx)), 1)
    idx += [0] * (l_size - len(idx))
    t_poly = vector_to_polynomial(table)
    i_poly = vector_to_polynomial(idx)
    g1 = params["g1_powers"]
    C_t = kzg_commit(g1, t_poly)
    C_i = kzg_commit(g1, i_poly)
    log_l = _log2_exact(l_size)
    tr = Transcript(params["fiat_shamir_seed"])
    tr.append_field_element(b"table_commitment", commitment_hash(C_t))
    tr.append_field_element(b"index_commitment", commitment_hash(C_i))
    i_mle = mle_from_evaluations_vec(log_l, idx)
    last = []

    def lookup_poly(vars_):  # src/shout.rs:166-183
        if len(vars_) != log_l:
            return 0
        last.append(mle_evaluate(i_mle, vars_))
        return 0

    rounds, final, chals = sumcheck_prove(log_l, 0, lookup_poly, tr)
    opening = tr.challenge_field_elements(b"opening_challenges", log_l)
    openings, finals = [], []
    if opening:
        z = opening[0]
        vt, pt = kzg_open(g1, t_poly, z)
        vi, pi = kzg_open(g1, i_poly, z)
        openings = [pt, pi]
        finals = [vt, vi]
    return dict(table_commitment=C_t, index_commitment=C_i,
                round_polynomials=rounds, final_evaluation=final,
                opening_proofs=openings, final_evaluations=finals,
                sumcheck_challenges=chals,
                opening_point=opening[0] if opening else None,
                table_poly=t_poly, index_poly=i_poly)


# ----------------------------------------------------------------------------
# Size-independent checks (test helpers, not part of the reference algorithm)
# ----------------------------------------------------------------------------
def barycentric_eval(ys, z: int) -> int:
    """Value at z of the interpolant of ys on nodes 0..n-1, in O(n) (no coefficients).

    f(z) = M(z) * sum_i y_i w_i / (z - i),  w_i = (-1)^(n-1-i) / (i! (n-1-i)!),
    M(z) = prod_i (z - i); if z is a node, f(z) = y_z.  Used to check commitments
    (z = tau) and openings at sizes the O(n^3) restatement cannot reach.
    """
    n = len(ys)
    z %= R_MOD
    if z < n:
        return ys[z] % R_MOD
    fact = [1] * n
    for i in range(1, n):
        fact[i] = fact[i - 1] * i % R_MOD
    inv_fact_last = fr_inv(fact[n - 1])
    inv_fact = [1] * n
    inv_fact[n - 1] = inv_fact_last
    for i in range(n - 1, 0, -1):
        inv_fact[i - 1] = inv_fact[i] * i % R_MOD
    # batch inverse of (z - i)
    d = [(z - i) % R_MOD for i in range(n)]
    pre = [1] * (n + 1)
    for i in range(n):
        pre[i + 1] = pre[i] * d[i] % R_MOD
    inv_all = fr_inv(pre[n])
    M = pre[n]
    acc = 0
    for i in range(n - 1, -1, -1):
        di_inv = inv_all * pre[i] % R_MOD
        inv_all = inv_all * d[i] % R_MOD
        if ys[i] % R_MOD:
            w = inv_fact[i] * inv_fact[n - 1 - i] % R_MOD
            if (n - 1 - i) & 1:
                w = R_MOD - w
            acc = (acc + ys[i] * w % R_MOD * di_inv) % R_MOD
    return acc * M % R_MOD


# ----------------------------------------------------------------------------
# BN254 pairing and the verifiers (src/commitments.rs:201-301, src/sumcheck.rs:113-150,
# src/twist.rs:255-304, src/shout.rs:225-274; arkworks Bn254::pairing).  Restated in a
# different representation from the product (csrc/pairing.cpp uses the Fq2/Fq6/Fq12 tower):
# Fq12 = Fq[w] / (w^12 - 18 w^6 + 82), with u = w^6 - 9 (so u^2 = -1) and G2 on the D-type
# twist y^2 = x^3 + 3/(9+u), untwisted by (x, y) -> (x w^2, y w^3).  The reduced optimal ate
# pairing f_{6x+2,Q}(P) l_{T,pi Q}(P) l_{T+pi Q,-pi^2 Q}(P) ^ ((p^12-1)/r) is unique.
# ----------------------------------------------------------------------------
BN_X = 4965661367192848881
G2_GEN = ((10857046999023057135944570762232829481370756359578518086990519993285655852781,
           11559732032986387107991004021392285783925812861821192530917403151452391805634),
          (8495653923123431417604973247489272438418190587263600148770280649306958101930,
           4082367875863433681332203403145435568316851327593401208105741076214120093531))


def _f12_mul(a, b):
    p = P_MOD
    t = [0] * 23
    for i, x in enumerate(a):
        if x:
            for j, y in enumerate(b):
                t[i + j] += x * y
    for k in range(22, 11, -1):  # w^12 = 18 w^6 - 82
        c = t[k]
        if c:
            t[k - 6] += 18 * c
            t[k - 12] -= 82 * c
    return [x % p for x in t[:12]]


def _f12_one():
    return [1] + [0] * 11


def _f12_pow(a, e):
    r = _f12_one()
    for bit in bin(e)[2:]:
        r = _f12_mul(r, r)
        if bit == "1":
            r = _f12_mul(r, a)
    return r


def _f12_inv(a):
    # a^(p^12 - 2) (Fermat in the field Fq12)
    return _f12_pow(a, P_MOD ** 12 - 2)


def _f12_from_fq2(a, shift):
    """(a0 + a1 u) * w^shift with u = w^6 - 9."""
    r = [0] * 12
    r[shift % 12] = (a[0] - 9 * a[1]) % P_MOD
    r[(shift + 6) % 12] = a[1] % P_MOD
    return r


def _untwist(Q):
    return (_f12_from_fq2(Q[0], 2), _f12_from_fq2(Q[1], 3))


def _f12_add(a, b):
    return [(x + y) % P_MOD for x, y in zip(a, b)]


def _f12_sub(a, b):
    return [(x - y) % P_MOD for x, y in zip(a, b)]


def _line(T, S, P, tangent):
    if tangent:
        x2 = _f12_mul(T[0], T[0])
        lam = _f12_mul([3 * v % P_MOD for v in x2], _f12_inv([2 * v % P_MOD for v in T[1]]))
    else:
        lam = _f12_mul(_f12_sub(S[1], T[1]), _f12_inv(_f12_sub(S[0], T[0])))
    l = _f12_sub(_f12_sub(P[1], T[1]), _f12_mul(lam, _f12_sub(P[0], T[0])))
    x3 = _f12_sub(_f12_sub(_f12_mul(lam, lam), T[0]), S[0])
    y3 = _f12_sub(_f12_mul(lam, _f12_sub(T[0], x3)), T[1])
    return l, (x3, y3)


def pairing(P, Q):
    """Reduced optimal ate pairing e(P, Q) (flat Fq12 coefficient list); P affine G1 or None,
    Q = ((x0, x1), (y0, y1)) on the twist or None."""
    if P is None or Q is None:
        return _f12_one()
    q = _untwist(Q)
    Pf = ([P[0] % P_MOD] + [0] * 11, [P[1] % P_MOD] + [0] * 11)
    f, T = _f12_one(), q
    for bit in bin(6 * BN_X + 2)[3:]:
        l, T = _line(T, T, Pf, True)
        f = _f12_mul(_f12_mul(f, f), l)
        if bit == "1":
            l, T = _line(T, q, Pf, False)
            f = _f12_mul(f, l)
    q1 = (_f12_pow(q[0], P_MOD), _f12_pow(q[1], P_MOD))
    q2 = (_f12_pow(q1[0], P_MOD), [(-v) % P_MOD for v in _f12_pow(q1[1], P_MOD)])
    l, T = _line(T, q1, Pf, False)
    f = _f12_mul(f, l)
    l, T = _line(T, q2, Pf, False)
    f = _f12_mul(f, l)
    return _f12_pow(f, (P_MOD ** 12 - 1) // R_MOD)


def tower_to_flat(c):
    """Product layout (12 Fq: c0.c0.c0, c0.c0.c1, ..., c1.c2.c1 of Fq12 = Fq6[w]/(w^2 - v),
    Fq6 = Fq2[v]/(v^3 - xi)) -> flat coefficients in w (v = w^2, u = w^6 - 9)."""
    r = [0] * 12
    for i in range(2):          # w^i
        for j in range(3):      # v^j = w^(2j)
            a0, a1 = c[6 * i + 2 * j], c[6 * i + 2 * j + 1]
            for k, v in enumerate(_f12_from_fq2((a0, a1), i + 2 * j)):
                r[k] = (r[k] + v) % P_MOD
    return r


# G2 arithmetic on the twist (Fq2 pairs), for the verifying key and batch verification
def _f2_mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P_MOD, (a[0] * b[1] + a[1] * b[0]) % P_MOD)


def _f2_inv(a):
    n = pow((a[0] * a[0] + a[1] * a[1]) % P_MOD, P_MOD - 2, P_MOD)
    return (a[0] * n % P_MOD, (-a[1]) * n % P_MOD)


def g2_add(A, B):
    if A is None:
        return B
    if B is None:
        return A
    if A[0] == B[0]:
        if A[1] != B[1] or A[1] == (0, 0):
            return None
        x2 = _f2_mul(A[0], A[0])
        lam = _f2_mul(((3 * x2[0]) % P_MOD, (3 * x2[1]) % P_MOD), _f2_inv(((2 * A[1][0]) % P_MOD, (2 * A[1][1]) % P_MOD)))
    else:
        lam = _f2_mul(((B[1][0] - A[1][0]) % P_MOD, (B[1][1] - A[1][1]) % P_MOD),
                      _f2_inv(((B[0][0] - A[0][0]) % P_MOD, (B[0][1] - A[0][1]) % P_MOD)))
    l2 = _f2_mul(lam, lam)
    x3 = ((l2[0] - A[0][0] - B[0][0]) % P_MOD, (l2[1] - A[0][1] - B[0][1]) % P_MOD)
    t = _f2_mul(lam, ((A[0][0] - x3[0]) % P_MOD, (A[0][1] - x3[1]) % P_MOD))
    return (x3, ((t[0] - A[1][0]) % P_MOD, (t[1] - A[1][1]) % P_MOD))


def g2_neg(A):
    return None if A is None else (A[0], ((-A[1][0]) % P_MOD, (-A[1][1]) % P_MOD))


def g2_mul(A, k):
    r = None
    for bit in bin(k % R_MOD)[2:] if k % R_MOD else "":
        r = g2_add(r, r)
        if bit == "1":
            r = g2_add(r, A)
    return r


def verifier_key(params):
    """CommitmentVerificationKey (src/utils.rs:104-112): (G1, G2, tau G2)."""
    return dict(g1=G1_GEN, g2=G2_GEN, g2_tau=g2_mul(G2_GEN, params["tau"]))


def kzg_verify(vk, C, z, v, proof):  # src/commitments.rs:201-228
    left = affine_add(C, g1_neg(affine_mul(vk["g1"], v))) if C is not None else g1_neg(affine_mul(vk["g1"], v))
    right = g2_add(vk["g2_tau"], g2_neg(g2_mul(vk["g2"], z)))
    return pairing(left, vk["g2"]) == pairing(proof, right)


def kzg_batch_verify(vk, Cs, zs, vs, proofs):  # src/commitments.rs:230-301, as written
    if not (len(Cs) == len(zs) == len(vs) == len(proofs)):
        raise ValueError("Batch verify input lengths must match")
    if not Cs:
        return True
    rng = ChaCha20Rng(bytes([42] * 32))
    gam = [fr_rand(rng) for _ in Cs]
    bc = bp = bg2 = None
    bv = 0
    for C, z, v, pi, g in zip(Cs, zs, vs, proofs, gam):
        bc = affine_add(bc, affine_mul(C, g)) if bc is not None else affine_mul(C, g)
        bv = (bv + v * g) % R_MOD
        bp = affine_add(bp, affine_mul(pi, g)) if bp is not None else affine_mul(pi, g)
        bg2 = g2_add(bg2, g2_mul(g2_add(vk["g2_tau"], g2_neg(g2_mul(vk["g2"], z))), g))
    left = affine_add(bc, g1_neg(affine_mul(vk["g1"], bv))) if bc is not None else g1_neg(affine_mul(vk["g1"], bv))
    return pairing(left, vk["g2"]) == pairing(bp, bg2)


def sumcheck_verify(rounds, final_eval, transcript):  # src/sumcheck.rs:113-150 (claimed 0)
    cur = 0
    for r, c in enumerate(rounds):
        if (horner_eval(c, 0) + horner_eval(c, 1)) % R_MOD != cur:
            return False
        transcript.append_field_elements(f"sumcheck_round_{r}".encode(), c)
        ch = transcript.challenge_field_element(f"sumcheck_challenge_{r}".encode())
        cur = horner_eval(c, ch)
    return cur == final_eval % R_MOD


def protocol_verify(vk, seed, labels, C, rounds, final_eval, openings, values):
    """Twist::verify (labels address/value) / Shout::verify (labels table/index)."""
    tr = Transcript(seed)
    tr.append_field_element(labels[0], commitment_hash(C[0]))
    tr.append_field_element(labels[1], commitment_hash(C[1]))
    if not sumcheck_verify(rounds, final_eval, tr):
        return False
    z = tr.challenge_field_elements(b"opening_challenges", len(rounds))
    if z and len(openings) >= 2 and len(values) >= 2:
        for k in range(2):
            if not kzg_verify(vk, C[k], z[0], values[k], openings[k]):
                return False
    return True


# ----------------------------------------------------------------------------
# Canonical serialisation (ark-serialize 0.4.2 / ark-ec 0.4.2 short-Weierstrass Affine,
# used by src/commitments.rs:94-154): x (and y) little-endian, SWFlags in the top bits of
# the last byte: YIsNegative = 0x80 (y > -y), PointAtInfinity = 0x40.
# ----------------------------------------------------------------------------
def g1_serialize(P, compressed=True):
    n = 32 if compressed else 64
    if P is None:
        out = bytearray(n)
        out[-1] |= 0x40
        return bytes(out)
    x, y = P
    out = bytearray(x.to_bytes(32, "little") + (b"" if compressed else y.to_bytes(32, "little")))
    if y > (P_MOD - y) % P_MOD:
        out[-1] |= 0x80
    return bytes(out)


def fr_serialize(x):
    return (x % R_MOD).to_bytes(32, "little")


def proof_serialize(commitments, rounds, final_eval, openings, finals, compressed=True):
    """Twist/ShoutProof fields in declaration order; Vec<T> = u64 LE length + elements."""
    u64 = lambda v: int(v).to_bytes(8, "little")  # noqa: E731
    out = b"".join(g1_serialize(C, compressed) for C in commitments)
    out += u64(len(rounds)) + b"".join(u64(len(r)) + b"".join(fr_serialize(c) for c in r) for r in rounds)
    out += fr_serialize(final_eval)
    out += u64(len(openings)) + b"".join(g1_serialize(P, compressed) for P in openings)
    out += u64(len(finals)) + b"".join(fr_serialize(v) for v in finals)
    return out
