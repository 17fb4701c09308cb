// f29.hpp -- BN254 Fq in radix 2^29: an accumulation variant measured in round 3 and NOT in the
// product (tools/mad29bench.hip, tests/test_f29_host.py; DESIGN.md §2.6 has the numbers: 14-20 %
// more mixed additions per second in isolation, no gain inside k_accumulate).
//
// 9 limbs of 29 bits, Montgomery form with R' = 2^261.  A column of the product-scanning
// Montgomery product sums at most 18 products of limbs below 2^30 x 2^29 (or 2^29 x 2^29 for the
// two-product form) plus the previous column's carry, which stays below 2^64: every multiply-add
// is ONE v_mad_u64_u32 into a 64-bit register pair -- no carry instruction per MAC -- and a column
// ends with one 64-bit shift (the pair stays where it is: no register rotation).  The radix-2^32
// product (mont_mul.inc) needs a carry instruction per MAC and a move per column; per mixed
// addition this form issues about a third fewer instructions, and k_accumulate is bound by its
// instruction count.
//
// Values are lazy: products return normalized limbs (< 2^29) and a value below about 1.7 M for
// inputs below 10 M (M / R' ~ 2^-7.36); subtractions add a multiple of M written with every limb
// >= the subtrahend's limbs (no borrows) and are renormalized where a product needs it.  Each
// bound is stated at its use in xyzz_madd29.  (It served k_accumulate's table plans through
// R'-form window tables in the measured build.)
#pragma once
#include "../multilinear-map-cryptography_amd/csrc/bn254.hpp"

namespace tns {

struct F29 {
  u32 v[9];
};

constexpr u32 F29_MASK = (1u << 29) - 1;
constexpr u32 F29_PINV = 0x04866389u;  // -M^{-1} mod 2^29 (Fq)

// the normalized radix-2^29 digits of k M (k small), at compile time
struct F29Digits {
  u32 d[9];
};
constexpr F29Digits f29_kM(unsigned k) {
  // M in 32-bit limbs (FqCfg::M) -> k M in 64-bit chunks -> 29-bit digits
  u64 w[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  u64 carry = 0;
  for (int i = 0; i < 8; i++) {
    const u64 t = (u64)FqCfg::M[i] * k + carry;
    w[i] = t & 0xffffffffull;
    carry = t >> 32;
  }
  w[8] = carry;
  F29Digits r{};
  for (int j = 0; j < 9; j++) {
    const int bit = 29 * j, limb = bit >> 5, sh = bit & 31;
    u64 x = w[limb] >> sh;
    if (sh > 3 && limb + 1 < 9) x |= w[limb + 1] << (32 - sh);
    r.d[j] = (u32)(x & F29_MASK);
  }
  return r;
}
// k M with every limb in [c (2^29 - 1), (c + 1) 2^29) but the top one, which is k M's top digit
// minus c: subtracting up to c normalized values limb by limb never borrows as long as their
// top digits sum to at most that -- k M must exceed the subtrahend by a margin (k = 2 for a
// canonical y: with k = 1 a y whose top digit equals M's left a negative top limb, the bug the
// SRS-table chains of tools/mad29bench-style checks missed and the skewed-MSM tests caught)
constexpr F29Digits f29_kM_offset(unsigned k, unsigned c) {
  F29Digits d = f29_kM(k), r{};
  for (int i = 0; i < 8; i++) r.d[i] = d.d[i] + c * (1u << 29) - (i ? c : 0u);
  r.d[8] = d.d[8] - c;
  return r;
}

template <unsigned K, unsigned C>
struct F29Const {
  static constexpr F29Digits v = f29_kM_offset(K, C);
};
struct F29M {
  static constexpr F29Digits v = f29_kM(1);
};

__device__ __forceinline__ void f29_normalize(F29 &a) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a.v[i + 1] += a.v[i] >> 29;
    a.v[i] &= F29_MASK;
  }
}

// Montgomery product, product scanning; a limbs < 2^30 (or < 2^31 when b is normalized),
// b limbs < 2^30; result normalized, value < a b / 2^261 + M
__device__ __forceinline__ F29 f29_mul(const F29 &a, const F29 &b) {
  u32 m[9];
  F29 r;
  u64 acc = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
#pragma unroll
    for (int i = (k > 8 ? k - 8 : 0); i <= (k < 8 ? k : 8); i++) acc += (u64)a.v[i] * b.v[k - i];
    if (k < 9) {
#pragma unroll
      for (int i = 0; i < k; i++) acc += (u64)m[i] * F29M::v.d[k - i];
      m[k] = ((u32)acc * F29_PINV) & F29_MASK;
      acc += (u64)m[k] * F29M::v.d[0];
    } else {
#pragma unroll
      for (int i = k - 8; i < 9; i++) acc += (u64)m[i] * F29M::v.d[k - i];
      r.v[k - 9] = (u32)acc & F29_MASK;
    }
    acc >>= 29;
  }
  r.v[8] = (u32)acc;
  return r;
}

// Montgomery square: each cross product once against a doubled limb; a limbs < 2^30
__device__ __forceinline__ F29 f29_sqr(const F29 &a) {
  u32 m[9], d[9];
#pragma unroll
  for (int i = 0; i < 9; i++) d[i] = a.v[i] << 1;
  F29 r;
  u64 acc = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
#pragma unroll
    for (int i = (k > 8 ? k - 8 : 0); 2 * i < k; i++) acc += (u64)a.v[i] * d[k - i];
    if ((k & 1) == 0) acc += (u64)a.v[k / 2] * a.v[k / 2];
    if (k < 9) {
#pragma unroll
      for (int i = 0; i < k; i++) acc += (u64)m[i] * F29M::v.d[k - i];
      m[k] = ((u32)acc * F29_PINV) & F29_MASK;
      acc += (u64)m[k] * F29M::v.d[0];
    } else {
#pragma unroll
      for (int i = k - 8; i < 9; i++) acc += (u64)m[i] * F29M::v.d[k - i];
      r.v[k - 9] = (u32)acc & F29_MASK;
    }
    acc >>= 29;
  }
  r.v[8] = (u32)acc;
  return r;
}

// (a b + c d) / 2^261 under ONE reduction; all four normalized (18 products of < 2^58 per
// column, plus the reduction's 9 of < 2^58: < 2^63)
__device__ __forceinline__ F29 f29_mul2(const F29 &a, const F29 &b, const F29 &c, const F29 &e) {
  u32 m[9];
  F29 r;
  u64 acc = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
#pragma unroll
    for (int i = (k > 8 ? k - 8 : 0); i <= (k < 8 ? k : 8); i++) {
      acc += (u64)a.v[i] * b.v[k - i];
      acc += (u64)c.v[i] * e.v[k - i];
    }
    if (k < 9) {
#pragma unroll
      for (int i = 0; i < k; i++) acc += (u64)m[i] * F29M::v.d[k - i];
      m[k] = ((u32)acc * F29_PINV) & F29_MASK;
      acc += (u64)m[k] * F29M::v.d[0];
    } else {
#pragma unroll
      for (int i = k - 8; i < 9; i++) acc += (u64)m[i] * F29M::v.d[k - i];
      r.v[k - 9] = (u32)acc & F29_MASK;
    }
    acc >>= 29;
  }
  r.v[8] = (u32)acc;
  return r;
}

// a + K - b limb by limb (K: a multiple of M from F29Const<k, c>, every limb >= b's); not normalized
template <class KC>
__device__ __forceinline__ F29 f29_sub(const F29 &a, const F29 &b) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = a.v[i] + KC::v.d[i] - b.v[i];
  return r;
}

// 8 x 32-bit limbs (a value < 2^256) <-> 9 x 29-bit limbs (same value)
__device__ __forceinline__ F29 f29_from32(const Fq &x) {
  F29 r;
#pragma unroll
  for (int j = 0; j < 9; j++) {
    const int bit = 29 * j, limb = bit >> 5, sh = bit & 31;
    const u32 lo = x.v[limb], hi = limb + 1 < 8 ? x.v[limb + 1] : 0u;
    const u32 w = sh ? (u32)((((u64)hi << 32) | lo) >> sh) : lo;
    r.v[j] = w & F29_MASK;
  }
  return r;
}
__device__ __forceinline__ Fq f29_to32(const F29 &a) {  // a normalized, value < 2^256
  Fq r;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int bit = 32 * i, j = bit / 29, sh = bit % 29;
    u64 x = (u64)a.v[j] >> sh;
    if (j + 1 < 9) x |= (u64)a.v[j + 1] << (29 - sh);
    if (j + 2 < 9 && 58 - sh < 32) x |= (u64)a.v[j + 2] << (58 - sh);
    r.v[i] = (u32)x;
  }
  return r;
}

struct G1Xyzz29 {
  F29 x, y, zz, zzz;
};

// constants as radix-2^29 digits (printed by python: digits of pow(2, e, M)):
// 2^256 mod M: f29_mul(X', C256) = X' 2^256 / 2^261 -- an R' = 2^261 value back in the R = 2^256
// form of bn254.hpp (value < 1.1 M: lazy, < 2M); 2^266 mod M: f29_mul(x, C266) = x 2^5, an R
// value in the R' form; 2^261 mod M: one in the R' form
struct F29C256 {
  static constexpr F29Digits v = {{0x058f0d9du, 0x1aea1c6eu, 0x11c2cf74u, 0x11d651ebu, 0x1462c0a7u, 0x11b7bc3cu,
                                   0x1cbd99bau, 0x183340fbu, 0x000e0a77u}};
};
struct F29C266 {
  static constexpr F29Digits v = {{0x13349ca1u, 0x1a5d84a8u, 0x0a3e5cacu, 0x100249e0u, 0x12b951e8u, 0x0e92d304u,
                                   0x14cb95b3u, 0x041b9d3du, 0x00058003u}};
};
struct F29One {
  static constexpr F29Digits v = {{0x157ccc21u, 0x141c2758u, 0x185230d3u, 0x014c0419u, 0x0aa36fb9u, 0x1d4240ceu,
                                   0x11d54c07u, 0x052ac7a8u, 0x000dc836u}};
};
template <class D>
__device__ __forceinline__ F29 f29_const() {
  F29 c;
#pragma unroll
  for (int i = 0; i < 9; i++) c.v[i] = D::v.d[i];
  return c;
}

__device__ __forceinline__ Fq f29_out(const F29 &a) {  // R' value (< 10 M) -> lazy R value (< 1.1 M)
  return f29_to32(f29_mul(a, f29_const<F29C256>()));
}
__device__ __forceinline__ F29 f29_in(const Fq &a) {  // R value (< 2^256) -> R' value (< 1.1 M)
  return f29_mul(f29_from32(a), f29_const<F29C266>());
}

__device__ __forceinline__ bool f29_eq_digits(const F29 &a, const F29Digits &d) {
  u32 x = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) x |= a.v[i] ^ d.d[i];
  return x == 0;
}

// the full comparison behind f29_is_kM's filter, out of line: inlined, the compiler if-converted
// its 81 limb compares into every addition (~250 instructions of a ~1 950-instruction madd)
__device__ __attribute__((noinline)) bool f29_is_kM_full(const F29 &p) {
  bool hit = false;
#pragma unroll
  for (unsigned k = 1; k <= 9; k++) hit |= f29_eq_digits(p, f29_kM(k));
  return hit;
}

// P (normalized, 0 < P < 10 M) a multiple of M?  A filter on the low limb first (one compare per
// candidate), the full comparison only when a low limb matches.
__device__ __forceinline__ bool f29_is_kM(const F29 &p) {
  bool cand = false;
#pragma unroll
  for (unsigned k = 1; k <= 9; k++) cand |= p.v[0] == f29_kM(k).d[0];
  if (__builtin_expect(!cand, 1)) return false;
  return f29_is_kM_full(p);
}

// XYZZ += affine in R' (k_accumulate's table plans; the formulas and order of xyzz_madd_lazy).
// Invariants of the running sum on entry and exit: all coordinates normalized, X < 7.7 M,
// Y < 2 M, ZZ, ZZZ < 1.7 M; `empty` stands for the identity (no coordinate is read).  q: canonical
// (< M) R' coordinates from the window table; neg: add -q.  The bounds below use
// eps = M / 2^261 < 0.0060 (a product of inputs < A M and < B M is < (A B eps + 1) M).
#ifdef TNS_F29_NOINLINE  // (debug builds)
__device__ __attribute__((noinline)) void xyzz_madd29(G1Xyzz29 &p, bool &empty, const F29 &x2, const F29 &y2, bool neg) {
#else
__device__ __forceinline__ void xyzz_madd29(G1Xyzz29 &p, bool &empty, const F29 &x2, const F29 &y2, bool neg) {
#endif
  const F29 y2n = f29_sub<F29Const<2, 1>>(F29{}, y2);  // 2M - y2 in (M, 2M), limbs < 2^30
  F29 yq;
#pragma unroll
  for (int i = 0; i < 9; i++) yq.v[i] = neg ? y2n.v[i] : y2.v[i];
  if (empty) {
    p.x = x2;
    p.y = yq;
    f29_normalize(p.y);
    p.zz = p.zzz = f29_const<F29One>();
    empty = false;
    return;
  }
  const F29 U2 = f29_mul(x2, p.zz);                                 // < 1.02 M
  const F29 S2 = f29_mul(yq, p.zzz);                                // yq < 2M: < 1.03 M
  F29 P = f29_sub<F29Const<8, 1>>(U2, p.x);                         // U2 + 8M - X1 in (0.3, 9.02) M
  f29_normalize(P);
  F29 R = f29_sub<F29Const<2, 1>>(S2, p.y);                         // (0, 3.03) M
  f29_normalize(R);
  if (f29_is_kM(P)) {  // U2 == X1: q = +-(the running sum) (rare)
    bool r0 = false;
#pragma unroll
    for (unsigned k = 1; k <= 3; k++) r0 |= f29_eq_digits(R, f29_kM(k));
    if (!r0) {  // q = -sum: the identity
      empty = true;
      return;
    }
    // q = sum: mdbl-2008-s-1 of q (bn254.hpp xyzz_mdbl) in R'
    F29 U = yq;
    f29_normalize(U);
#pragma unroll
    for (int i = 0; i < 9; i++) U.v[i] <<= 1;                      // 2y < 2M, limbs < 2^30
    const F29 V = f29_sqr(U), W = f29_mul(U, V), S = f29_mul(x2, V);
    const F29 X2 = f29_sqr(x2);
    F29 M3;
#pragma unroll
    for (int i = 0; i < 9; i++) M3.v[i] = 3 * X2.v[i];              // < 3.1 M, limbs < 2^31
    f29_normalize(M3);
    F29 S2x;
#pragma unroll
    for (int i = 0; i < 9; i++) S2x.v[i] = 2 * S.v[i];              // 2S, limbs < 2^30
    F29 X3 = f29_sub<F29Const<3, 2>>(f29_sqr(M3), S2x);             // M3^2 + 3M - 2S in (0.9, 4.1) M
    f29_normalize(X3);
    F29 SX = f29_sub<F29Const<5, 1>>(S, X3);                        // S + 5M - X3 in (0.9, 6.1) M
    f29_normalize(SX);
    F29 yqn = yq;
    f29_normalize(yqn);
    F29 Wn = f29_sub<F29Const<2, 1>>(F29{}, W);                     // 2M - W in (0.9, 2) M
    f29_normalize(Wn);
    p.x = X3;
    p.y = f29_mul2(M3, SX, Wn, yqn);                                // M3 (S - X3) - W y
    p.zz = V;
    p.zzz = W;
    return;
  }
  const F29 PP = f29_sqr(P);                                        // < 1.49 M
  const F29 PPP = f29_mul(P, PP);                                   // < 1.09 M
  p.zz = f29_mul(p.zz, PP);                                         // < 1.02 M
  p.zzz = f29_mul(p.zzz, PPP);                                      // < 1.02 M
  const F29 Q = f29_mul(p.x, PP);                                   // < 1.07 M
  F29 t;
#pragma unroll
  for (int i = 0; i < 9; i++) t.v[i] = PPP.v[i] + 2 * Q.v[i];       // PPP + 2Q < 3.23 M, limbs < 3 2^29
  F29 X3 = f29_sub<F29Const<4, 3>>(f29_sqr(R), t);                  // R^2 + 4M - PPP - 2Q in (0.77, 5.06) M
  f29_normalize(X3);
  F29 QX = f29_sub<F29Const<6, 1>>(Q, X3);                          // Q + 6M - X3 in (0.94, 7.07) M
  f29_normalize(QX);
  F29 Pn = f29_sub<F29Const<2, 1>>(F29{}, PPP);                     // 2M - PPP in (0.91, 2) M
  f29_normalize(Pn);
  p.y = f29_mul2(R, QX, p.y, Pn);                                   // R (Q - X3) - Y1 PPP: < 1.16 M
  p.x = X3;
}

}  // namespace tns
