// bn254.hpp -- BN254 Fr / Fq Montgomery arithmetic and G1 group law for gfx950 (and host).
//
// Layout: a field element is 8 x u32 little-endian limbs in Montgomery form with
// R = 2^256 -- byte-identical to arkworks' `Fp256` ([u64; 4] Montgomery), so
// buffers cross the C ABI without conversion (src/utils.rs:14 FieldElement = ark_bn254::Fr).
//
// Multiplication is CIOS Montgomery with the "no-carry" shortcut (the top limb of
// both moduli is < 2^31 - 1), built on 32x32+64 -> 64 multiply-adds, which hipcc
// lowers to v_mad_u64_u32 on CDNA4.
//
// G1: y^2 = x^3 + 3 over Fq (ark-bn254 0.4.0).  Bucket sums use XYZZ coordinates
// (x = X/ZZ, y = Y/ZZZ; identity <=> ZZ == 0), affine SRS points are (x, y) with
// the all-zero pair standing for the identity.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define TNS_HD __host__ __device__ __forceinline__
#define TNS_DEV __device__ __forceinline__
#else
#define TNS_HD inline
#define TNS_DEV inline
#endif

namespace tns {

typedef uint32_t u32;
typedef uint64_t u64;

struct FrCfg {
  static constexpr u32 M[8] = {0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                               0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  static constexpr u32 ONE[8] = {0x4ffffffbu, 0xac96341cu, 0x9f60cd29u, 0x36fc7695u,
                                 0x7879462eu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
  static constexpr u32 R2[8] = {0xae216da7u, 0x1bb8e645u, 0xe35c59e3u, 0x53fe3ab1u,
                                0x53bb8085u, 0x8c49833du, 0x7f4e44a5u, 0x0216d0b1u};
  static constexpr u32 INV = 0xefffffffu;
  static constexpr u32 M2[8] = {0xe0000002u, 0x87c3eb27u, 0xf372e122u, 0x5067d090u,
                                0x0302b0bau, 0x70a08b6du, 0xc2634053u, 0x60c89ce5u};  // 2M
  static constexpr u32 R3[8] = {0xb4bf0040u, 0x5e94d8e1u, 0x1cfbb6b8u, 0x2a489cbeu,
                                0xa19fcfedu, 0x893cc664u, 0x7fcc657cu, 0x0cf8594bu};  // 2^768 mod M
};
struct FqCfg {
  static constexpr u32 M[8] = {0xd87cfd47u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                               0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  static constexpr u32 ONE[8] = {0xc58f0d9du, 0xd35d438du, 0xf5c70b3du, 0x0a78eb28u,
                                 0x7879462cu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
  static constexpr u32 R2[8] = {0x538afa89u, 0xf32cfc5bu, 0xd44501fbu, 0xb5e71911u,
                                0x0a417ff6u, 0x47ab1effu, 0xcab8351fu, 0x06d89f71u};
  static constexpr u32 INV = 0xe4866389u;
  static constexpr u32 M2[8] = {0xb0f9fa8eu, 0x7841182du, 0xd0e3951au, 0x2f02d522u,
                                0x0302b0bbu, 0x70a08b6du, 0xc2634053u, 0x60c89ce5u};  // 2M
  static constexpr u32 R3[8] = {0xda1530dfu, 0xb1cd6dafu, 0xa7283db6u, 0x62f210e6u,
                                0x0ada0afbu, 0xef7f0b0cu, 0x2d592544u, 0x20fd6e90u};  // 2^768 mod M
};

template <class C>
struct alignas(16) Fp {
  u32 v[8];

  TNS_HD static Fp zero() {
    Fp r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = 0;
    return r;
  }
  TNS_HD static Fp one() {
    Fp r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = C::ONE[i];
    return r;
  }
  TNS_HD bool is_zero() const {
    u32 acc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) acc |= v[i];
    return acc == 0;
  }
  TNS_HD bool operator==(const Fp &o) const {
    u32 acc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) acc |= v[i] ^ o.v[i];
    return acc == 0;
  }
  TNS_HD bool operator!=(const Fp &o) const { return !(*this == o); }
};

typedef Fp<FrCfg> Fr;
typedef Fp<FqCfg> Fq;

#if defined(__HIPCC__)
#if defined(TNS_FIELD_BI)
#include "field_bi.inc"
#else
#include "field_asm.inc"
#endif
#endif

// ---------------------------------------------------------------- raw 256-bit helpers
// r = a - M if a >= M (a < 2M assumed)
template <class C>
TNS_HD void reduce_once(Fp<C> &a) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(TNS_NO_FIELD_ASM)
  reduce_once_dev(a);
  return;
#endif
  u32 t[8];
  u64 br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    u64 d = (u64)a.v[i] - C::M[i] - br;
    t[i] = (u32)d;
    br = (d >> 32) & 1;
  }
  if (!br) {
#pragma unroll
    for (int i = 0; i < 8; i++) a.v[i] = t[i];
  }
}

template <class C>
TNS_HD Fp<C> add(const Fp<C> &a, const Fp<C> &b) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(TNS_NO_FIELD_ASM)
  return add_dev(a, b);
#endif
  Fp<C> r;
  u64 c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    c += (u64)a.v[i] + b.v[i];
    r.v[i] = (u32)c;
    c >>= 32;
  }
  reduce_once(r);  // a + b < 2M < 2^256: no carry out of limb 7
  return r;
}

template <class C>
TNS_HD Fp<C> sub(const Fp<C> &a, const Fp<C> &b) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(TNS_NO_FIELD_ASM)
  return sub_dev(a, b);
#endif
  Fp<C> r;
  u64 br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    u64 d = (u64)a.v[i] - b.v[i] - br;
    r.v[i] = (u32)d;
    br = (d >> 32) & 1;
  }
  if (br) {
    u64 c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      c += (u64)r.v[i] + C::M[i];
      r.v[i] = (u32)c;
      c >>= 32;
    }
  }
  return r;
}

template <class C>
TNS_HD Fp<C> neg(const Fp<C> &a) {
  if (a.is_zero()) return a;
  Fp<C> r;
  u64 br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    u64 d = (u64)C::M[i] - a.v[i] - br;
    r.v[i] = (u32)d;
    br = (d >> 32) & 1;
  }
  return r;
}

template <class C>
TNS_HD Fp<C> dbl(const Fp<C> &a) {
  return add(a, a);
}

#if defined(__HIPCC__)
#ifdef TNS_MONT_MUL_INC  // benchmark builds (tools/maddbench.hip) swap the product variant
#include TNS_MONT_MUL_INC
#else
#include "mont_mul.inc"
#endif
#endif

// Host (and reference): CIOS Montgomery product, no-carry variant (top modulus limb < 2^31 - 1).
template <class C>
TNS_HD Fp<C> mul_cios(const Fp<C> &a, const Fp<C> &b) {
  u32 t[8];
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const u32 bi = b.v[i];
    u64 A = (u64)a.v[0] * bi + t[0];
    const u32 m = (u32)A * C::INV;
    u64 Cc = (u64)m * C::M[0] + (u32)A;
#pragma unroll
    for (int j = 1; j < 8; j++) {
      A = (u64)a.v[j] * bi + ((u64)t[j] + (A >> 32));
      Cc = (u64)m * C::M[j] + ((u64)(u32)A + (Cc >> 32));
      t[j - 1] = (u32)Cc;
    }
    t[7] = (u32)((A >> 32) + (Cc >> 32));
  }
  Fp<C> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = t[i];
  reduce_once(r);
  return r;
}

#if !defined(__HIP_DEVICE_COMPILE__)
// Host: the same CIOS product on 4 x u64 limbs with 128-bit products (16 word products instead
// of 64): the prover's host-side group arithmetic between kernels (bucket-sum recombination,
// affine conversions, transcript hashing of commitments) runs ~3x faster.  Both forms use
// R = 2^256 and return the canonical representative, so results are identical.
template <class C>
struct Cfg64 {
  static constexpr u64 m(int i) { return (u64)C::M[2 * i] | ((u64)C::M[2 * i + 1] << 32); }
  static constexpr u64 inv() {  // -M^{-1} mod 2^64 (Newton)
    u64 x = 1;
    for (int i = 0; i < 7; i++) x *= 2 - m(0) * x;
    return (u64)0 - x;
  }
};

template <class C>
inline Fp<C> mul_cios64(const Fp<C> &a, const Fp<C> &b) {
  typedef unsigned __int128 u128;
  constexpr u64 M[4] = {Cfg64<C>::m(0), Cfg64<C>::m(1), Cfg64<C>::m(2), Cfg64<C>::m(3)};
  constexpr u64 INV = Cfg64<C>::inv();
  u64 x[4], y[4], t[4] = {0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    x[i] = (u64)a.v[2 * i] | ((u64)a.v[2 * i + 1] << 32);
    y[i] = (u64)b.v[2 * i] | ((u64)b.v[2 * i + 1] << 32);
  }
  for (int i = 0; i < 4; i++) {
    u128 s = (u128)x[0] * y[i] + t[0];
    u64 A = (u64)(s >> 64);
    const u64 t0 = (u64)s, m = t0 * INV;
    s = (u128)m * M[0] + t0;
    u64 Cc = (u64)(s >> 64);
    for (int j = 1; j < 4; j++) {
      s = (u128)x[j] * y[i] + t[j] + A;
      A = (u64)(s >> 64);
      s = (u128)m * M[j] + (u64)s + Cc;
      Cc = (u64)(s >> 64);
      t[j - 1] = (u64)s;
    }
    t[3] = Cc + A;
  }
  Fp<C> r;
  for (int i = 0; i < 4; i++) {
    r.v[2 * i] = (u32)t[i];
    r.v[2 * i + 1] = (u32)(t[i] >> 32);
  }
  reduce_once(r);
  return r;
}
#endif

template <class C>
TNS_HD Fp<C> mul(const Fp<C> &a, const Fp<C> &b) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(TNS_MUL_CIOS)
  return mul_ps_dev(a, b);
#elif defined(__HIP_DEVICE_COMPILE__)
  return mul_cios(a, b);
#else
  return mul_cios64(a, b);
#endif
}

template <class C>
TNS_HD Fp<C> sqr(const Fp<C> &a) {
  return mul(a, a);
}

// multiply by a small constant via additions
template <class C>
TNS_HD Fp<C> mul3(const Fp<C> &a) {
  return add(add(a, a), a);
}

template <class C>
TNS_HD Fp<C> to_mont(const Fp<C> &canonical) {
  Fp<C> r2;
#pragma unroll
  for (int i = 0; i < 8; i++) r2.v[i] = C::R2[i];
  return mul(canonical, r2);
}

template <class C>
TNS_HD Fp<C> from_mont(const Fp<C> &a) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(TNS_MUL_CIOS)
  return redc_dev(a);  // the reduction alone: a * 1 needs no product columns
#endif
  Fp<C> one = Fp<C>::zero();
  one.v[0] = 1;
  return mul(a, one);
}

template <class C>
TNS_HD Fp<C> from_u64(u64 x) {
  Fp<C> c = Fp<C>::zero();
  c.v[0] = (u32)x;
  c.v[1] = (u32)(x >> 32);
  return to_mont(c);
}

// a^e for a 256-bit exponent given as 8 limbs (square-and-multiply, MSB first)
template <class C>
TNS_HD Fp<C> pow_limbs(const Fp<C> &a, const u32 e[8]) {
  Fp<C> acc = Fp<C>::one();
  for (int i = 255; i >= 0; i--) {
    acc = sqr(acc);
    if ((e[i >> 5] >> (i & 31)) & 1) acc = mul(acc, a);
  }
  return acc;
}

template <class C>
TNS_HD Fp<C> pow_u64(const Fp<C> &a, u64 e) {
  Fp<C> acc = Fp<C>::one(), base = a;
  while (e) {
    if (e & 1) acc = mul(acc, base);
    base = sqr(base);
    e >>= 1;
  }
  return acc;
}

#if defined(__HIPCC__)
#include "inv_chain.inc"
// Device Fermat inverse: a^(M-2) along a sliding-window (3-bit) addition chain over the constant
// exponent (tools/gen_inv_chain.py: 62 window products for Fr, 56 for Fq, instead of the 127 /
// 130 single-bit products of square-and-multiply), squarings with the dedicated lazy square,
// everything in the lazy [0, 2M) domain until the final conditional subtraction.  The chain
// is read from constant memory with a uniform index: the walk is uniform control flow.
template <class C>
__device__ __forceinline__ Fp<C> inv_window_dev(const Fp<C> &a) {
  const Fp<C> a2 = sqr_lazy_dev(a);
  const Fp<C> t1 = a, t3 = mul_lazy_dev(a, a2), t5 = mul_lazy_dev(t3, a2), t7 = mul_lazy_dev(t5, a2);
  const unsigned char *steps = InvChain<C>::steps();
  auto entry = [&](unsigned idx) -> const Fp<C> & { return idx == 0 ? t1 : idx == 1 ? t3 : idx == 2 ? t5 : t7; };
  Fp<C> acc = entry(steps[0] & 3);
  for (int k = 1; k < InvChain<C>::n; k++) {
    const unsigned st = steps[k];
    for (unsigned q = 0; q < (st >> 2); q++) acc = sqr_lazy_dev(acc);
    acc = mul_lazy_dev(acc, entry(st & 3));
  }
  reduce_once(acc);  // lazy products of inputs < 2M stay < 2M
  return acc;
}
#endif

#if defined(__HIPCC__)
// Single inversions on a latency path (one thread of a block inverts while the others wait:
// k_chain_inv): the binary extended Euclid on the representation x = a R mod M, variable time
// (the inputs are public), x^-1 = a^-1 R^-1, then one Montgomery product with R^3 gives
// a^-1 R.  About 2 log2 M shift steps and log2 M subtractions of 8-limb words: ~4x fewer
// instructions than the Fermat chain's ~310 products.  Inverse of zero is zero.
template <class C>
__device__ __forceinline__ void limbs_half_mod(u32 (&x)[8]) {  // x / 2 mod M (x < M)
  if (x[0] & 1u) {  // x + M < 2^255: no carry out of the top limb
    u64 t = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      t += (u64)x[i] + C::M[i];
      x[i] = (u32)t;
      t >>= 32;
    }
  }
#pragma unroll
  for (int i = 0; i < 7; i++) x[i] = (x[i] >> 1) | (x[i + 1] << 31);
  x[7] >>= 1;
}
template <class C>
__device__ __forceinline__ void limbs_sub_mod(u32 (&x)[8], const u32 (&y)[8]) {  // x - y mod M (x, y < M)
  u64 br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const u64 d = (u64)x[i] - y[i] - br;
    x[i] = (u32)d;
    br = (d >> 32) & 1;
  }
  if (br) {
    u64 t = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      t += (u64)x[i] + C::M[i];
      x[i] = (u32)t;
      t >>= 32;
    }
  }
}
template <class C>
__device__ Fp<C> inv_binary_dev(const Fp<C> &a) {
  u32 u[8], v[8], x1[8], x2[8];
  u32 any = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    u[i] = a.v[i];
    v[i] = C::M[i];
    x1[i] = i == 0 ? 1u : 0u;
    x2[i] = 0;
    any |= a.v[i];
  }
  if (!any) return Fp<C>::zero();
  auto is_one = [](const u32(&w)[8]) {
    u32 hi = 0;
#pragma unroll
    for (int i = 1; i < 8; i++) hi |= w[i];
    return w[0] == 1u && hi == 0;
  };
  auto shr1 = [](u32(&w)[8]) {
#pragma unroll
    for (int i = 0; i < 7; i++) w[i] = (w[i] >> 1) | (w[i + 1] << 31);
    w[7] >>= 1;
  };
  auto geq = [](const u32(&x)[8], const u32(&y)[8]) {
    bool r = true, decided = false;
#pragma unroll
    for (int i = 7; i >= 0; i--) {
      if (!decided && x[i] != y[i]) {
        r = x[i] > y[i];
        decided = true;
      }
    }
    return r;
  };
  auto sub = [](u32(&x)[8], const u32(&y)[8]) {
    u64 br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const u64 d = (u64)x[i] - y[i] - br;
      x[i] = (u32)d;
      br = (d >> 32) & 1;
    }
  };
  while (!is_one(u) && !is_one(v)) {
    while (!(u[0] & 1u)) {
      shr1(u);
      limbs_half_mod<C>(x1);
    }
    while (!(v[0] & 1u)) {
      shr1(v);
      limbs_half_mod<C>(x2);
    }
    if (geq(u, v)) {
      sub(u, v);
      limbs_sub_mod<C>(x1, x2);
    } else {
      sub(v, u);
      limbs_sub_mod<C>(x2, x1);
    }
  }
  Fp<C> r, k;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    r.v[i] = is_one(u) ? x1[i] : x2[i];
    k.v[i] = C::R3[i];
  }
  return mul(r, k);  // (a R)^-1 R^3 R^-1 = a^-1 R
}
#endif

#if !defined(__HIP_DEVICE_COMPILE__)
// Host inverse by the binary extended Euclid on 4 x u64 limbs (~3x faster than the Fermat chain's
// ~380 products: the host inverts on the proof's critical path -- the commitments' and openings'
// affine forms, the barycentric batch inversion's one inverse).  a = xR (Montgomery limbs < M) ->
// r = (xR)^-1 mod M, and x^-1 R = mont(r, R^3).  Inverse of zero is zero.
template <class C>
inline Fp<C> inv_binary_host(const Fp<C> &a) {
  typedef unsigned __int128 u128;
  u64 u[4], v[4], x1[4] = {1, 0, 0, 0}, x2[4] = {0, 0, 0, 0}, m[4];
  for (int i = 0; i < 4; i++) {
    u[i] = (u64)a.v[2 * i] | ((u64)a.v[2 * i + 1] << 32);
    m[i] = (u64)C::M[2 * i] | ((u64)C::M[2 * i + 1] << 32);
    v[i] = m[i];
  }
  auto is_one = [](const u64 *w) { return w[0] == 1 && (w[1] | w[2] | w[3]) == 0; };
  auto shr1 = [](u64 *w) {
    for (int i = 0; i < 3; i++) w[i] = (w[i] >> 1) | (w[i + 1] << 63);
    w[3] >>= 1;
  };
  auto half_mod = [&](u64 *x) {  // x / 2 mod M (x < M < 2^255: x + M fits)
    if (x[0] & 1) {
      u64 c = 0;
      for (int i = 0; i < 4; i++) {
        const u128 t = (u128)x[i] + m[i] + c;
        x[i] = (u64)t;
        c = (u64)(t >> 64);
      }
    }
    shr1(x);
  };
  auto geq = [](const u64 *p, const u64 *q) {
    for (int i = 3; i >= 0; i--)
      if (p[i] != q[i]) return p[i] > q[i];
    return true;
  };
  auto sub_in = [](u64 *p, const u64 *q) {  // p -= q, returns the borrow
    u64 b = 0;
    for (int i = 0; i < 4; i++) {
      const u128 t = (u128)p[i] - q[i] - b;
      p[i] = (u64)t;
      b = (u64)(t >> 64) & 1;
    }
    return b;
  };
  auto sub_mod = [&](u64 *p, const u64 *q) {  // p = p - q mod M
    if (sub_in(p, q)) {
      u64 c = 0;
      for (int i = 0; i < 4; i++) {
        const u128 t = (u128)p[i] + m[i] + c;
        p[i] = (u64)t;
        c = (u64)(t >> 64);
      }
    }
  };
  while (geq(u, m)) sub_in(u, m);  // (a lazily reduced input: < 2M)
  if ((u[0] | u[1] | u[2] | u[3]) == 0) return Fp<C>::zero();
  while (!is_one(u) && !is_one(v)) {
    while ((u[0] & 1) == 0) {
      shr1(u);
      half_mod(x1);
    }
    while ((v[0] & 1) == 0) {
      shr1(v);
      half_mod(x2);
    }
    if (geq(u, v)) {
      sub_in(u, v);
      sub_mod(x1, x2);
    } else {
      sub_in(v, u);
      sub_mod(x2, x1);
    }
  }
  const u64 *r = is_one(u) ? x1 : x2;
  Fp<C> out, r2;
  for (int i = 0; i < 4; i++) {
    out.v[2 * i] = (u32)r[i];
    out.v[2 * i + 1] = (u32)(r[i] >> 32);
  }
  for (int i = 0; i < 8; i++) r2.v[i] = C::R2[i];
  static const Fp<C> r3 = mul_cios64(r2, r2);  // R^3 mod M
  return mul_cios64(out, r3);
}
#endif

// Fermat inverse (a^(M-2)) on the device; the binary extended Euclid on the host.  Inverse of
// zero is zero.
template <class C>
TNS_HD Fp<C> inv(const Fp<C> &a) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(TNS_MUL_CIOS)
  return inv_window_dev(a);
#endif
#if !defined(__HIP_DEVICE_COMPILE__)
  return inv_binary_host(a);
#endif
  u32 e[8];
  u64 br = 2;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    u64 d = (u64)C::M[i] - br;
    e[i] = (u32)d;
    br = (d >> 32) & 1;
  }
  return pow_limbs(a, e);
}

// canonical-integer comparison helpers (operate on from_mont'ed values)
template <class C>
TNS_HD bool geq_raw(const u32 a[8], const u32 b[8]) {
  for (int i = 7; i >= 0; i--) {
    if (a[i] > b[i]) return true;
    if (a[i] < b[i]) return false;
  }
  return true;
}

// ---------------------------------------------------------------- G1
struct alignas(16) G1Affine {  // identity <=> x == y == 0
  Fq x, y;
  TNS_HD bool is_inf() const { return x.is_zero() && y.is_zero(); }
};

struct alignas(16) G1Xyzz {  // identity <=> zz == 0
  Fq x, y, zz, zzz;
  TNS_HD static G1Xyzz inf() {
    G1Xyzz r;
    r.x = Fq::one();
    r.y = Fq::one();
    r.zz = Fq::zero();
    r.zzz = Fq::zero();
    return r;
  }
  TNS_HD bool is_inf() const { return zz.is_zero(); }
};

struct alignas(16) G1Jac {  // arkworks G1Projective layout (Jacobian); identity <=> z == 0
  Fq x, y, z;
};

TNS_HD G1Affine g1_neg(const G1Affine &p) {
  G1Affine r;
  r.x = p.x;
  r.y = neg(p.y);
  return r;
}

// dbl-2008-s-1 (a = 0)
TNS_HD G1Xyzz xyzz_dbl(const G1Xyzz &p) {
  if (p.is_inf() || p.y.is_zero()) return G1Xyzz::inf();
  Fq U = dbl(p.y);
  Fq V = sqr(U);
  Fq W = mul(U, V);
  Fq S = mul(p.x, V);
  Fq M = mul3(sqr(p.x));
  G1Xyzz r;
  r.x = sub(sqr(M), dbl(S));
  r.y = sub(mul(M, sub(S, r.x)), mul(W, p.y));
  r.zz = mul(V, p.zz);
  r.zzz = mul(W, p.zzz);
  return r;
}

// mdbl-2008-s-1: double an affine point
TNS_HD G1Xyzz xyzz_mdbl(const G1Affine &p) {
  if (p.is_inf() || p.y.is_zero()) return G1Xyzz::inf();
  Fq U = dbl(p.y);
  Fq V = sqr(U);
  Fq W = mul(U, V);
  Fq S = mul(p.x, V);
  Fq M = mul3(sqr(p.x));
  G1Xyzz r;
  r.x = sub(sqr(M), dbl(S));
  r.y = sub(mul(M, sub(S, r.x)), mul(W, p.y));
  r.zz = V;
  r.zzz = W;
  return r;
}

// madd-2008-s: XYZZ += affine
TNS_HD G1Xyzz xyzz_madd(const G1Xyzz &p, const G1Affine &q) {
  if (q.is_inf()) return p;
  if (p.is_inf()) {
    G1Xyzz r;
    r.x = q.x;
    r.y = q.y;
    r.zz = Fq::one();
    r.zzz = Fq::one();
    return r;
  }
  Fq U2 = mul(q.x, p.zz);
  Fq S2 = mul(q.y, p.zzz);
  Fq P = sub(U2, p.x);
  Fq R = sub(S2, p.y);
  if (P.is_zero()) {
    if (R.is_zero()) return xyzz_mdbl(q);
    return G1Xyzz::inf();
  }
  Fq PP = sqr(P);
  Fq PPP = mul(P, PP);
  Fq Q = mul(p.x, PP);
  G1Xyzz r;
  r.x = sub(sub(sqr(R), PPP), dbl(Q));
  r.y = sub(mul(R, sub(Q, r.x)), mul(p.y, PPP));
  r.zz = mul(p.zz, PP);
  r.zzz = mul(p.zzz, PPP);
  return r;
}

#if defined(__HIPCC__)
// ---- lazy-reduction mixed addition for the MSM accumulation (device only).  Coordinates of
// the running sum live in [0, 2M): products skip their final conditional subtraction
// (inputs < 2M give results < 2M since 4M < 2^256), sums and differences reduce against 2M,
// and "is zero mod M" is {0, M}.  The affine input is canonical; xyzz_canon brings a sum
// back to [0, M) before anything else reads it.
__device__ __forceinline__ bool fq_zero_lazy(const Fq &a) {
  u32 z = 0, m = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    z |= a.v[i];
    m |= a.v[i] ^ FqCfg::M[i];
  }
  return z == 0 || m == 0;
}

// K - a for a constant K >= a (no borrow out, no correction): K = M negates a canonical value,
// K = 2M forms the lazy-domain negation of a value in [0, 2M).  a is tied to the result (no
// early-clobber operand, see field_asm.inc); the borrow-chain limbs of K come from VGPRs (one
// constant-bus read per VALU instruction on gfx9: VCC is already one).
template <class C, bool TWO_M>
__device__ __forceinline__ Fp<C> const_minus_dev(const Fp<C> &a) {
#if defined(TNS_FIELD_BI)
  Fp<C> d;
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) d.v[i] = __builtin_subc(TWO_M ? C::M2[i] : C::M[i], a.v[i], br, &br);
  return d;
#endif
  Fp<C> r = a;
  const u32 *K = TWO_M ? C::M2 : C::M;
  asm("v_sub_co_u32_e32 %0, vcc, %8, %0\n\tv_subb_co_u32_e32 %1, vcc, %9, %1, vcc\n\t"
      "v_subb_co_u32_e32 %2, vcc, %10, %2, vcc\n\tv_subb_co_u32_e32 %3, vcc, %11, %3, vcc\n\t"
      "v_subb_co_u32_e32 %4, vcc, %12, %4, vcc\n\tv_subb_co_u32_e32 %5, vcc, %13, %5, vcc\n\t"
      "v_subb_co_u32_e32 %6, vcc, %14, %6, vcc\n\tv_subb_co_u32_e32 %7, vcc, %15, %7, vcc"
      : "+v"(r.v[0]), "+v"(r.v[1]), "+v"(r.v[2]), "+v"(r.v[3]), "+v"(r.v[4]), "+v"(r.v[5]), "+v"(r.v[6]), "+v"(r.v[7])
      : "s"(K[0]), "v"(K[1]), "v"(K[2]), "v"(K[3]), "v"(K[4]), "v"(K[5]), "v"(K[6]), "v"(K[7])
      : "vcc");
  return r;
}

__device__ __forceinline__ G1Xyzz xyzz_madd_lazy(const G1Xyzz &p, const G1Affine &q) {
  if (q.is_inf()) return p;
  if (p.is_inf()) {
    G1Xyzz r;
    r.x = q.x;
    r.y = q.y;
    r.zz = Fq::one();
    r.zzz = Fq::one();
    return r;
  }
  const Fq U2 = mul_lazy_dev(q.x, p.zz);
  const Fq S2 = mul_lazy_dev(q.y, p.zzz);
  const Fq P = sub2_dev(U2, p.x);
  const Fq R = sub2_dev(S2, p.y);
  if (fq_zero_lazy(P)) {
    if (fq_zero_lazy(R)) return xyzz_mdbl(q);
    return G1Xyzz::inf();
  }
  // ordered for register pressure: ZZ1, ZZZ1 die in ZZ3 / ZZZ3 right after PP / PPP, X1 and PP
  // in Q; the peak live set is PP, PPP, R, X1, Y1 and the two Z coordinates
  const Fq PP = sqr_lazy_dev(P);
  const Fq PPP = mul_lazy_dev(P, PP);
  G1Xyzz r;
  r.zz = mul_lazy_dev(p.zz, PP);
  r.zzz = mul_lazy_dev(p.zzz, PPP);
  const Fq Q = mul_lazy_dev(p.x, PP);
  r.x = sub2_dev(sub2_dev(sqr_lazy_dev(R), PPP), add2_dev(Q, Q));
  // Y3 = R (Q - X3) - Y1 PPP as ONE reduction of R (Q - X3) + Y1 (2M - PPP)  (PPP in [0, 2M))
  r.y = mul2_lazy_dev(R, sub2_dev(Q, r.x), p.y, const_minus_dev<FqCfg, true>(PPP));
  return r;
}

__device__ __forceinline__ G1Xyzz xyzz_canon(G1Xyzz p) {
  reduce_once_dev(p.x);
  reduce_once_dev(p.y);
  reduce_once_dev(p.zz);
  reduce_once_dev(p.zzz);
  return p;
}

// add-2008-s (XYZZ + XYZZ) in the lazy domain: both inputs in [0, 2M) (canonical points
// included), result in [0, 2M); the identity is zz in {0, M}.  The bucket fixup and the
// bucket reduction chain these; whatever the host reads goes through xyzz_canon first.
__device__ __forceinline__ G1Xyzz xyzz_add_lazy(const G1Xyzz &p, const G1Xyzz &q) {
  if (fq_zero_lazy(q.zz)) return p;
  if (fq_zero_lazy(p.zz)) return q;
  const Fq U1 = mul_lazy_dev(p.x, q.zz);
  const Fq U2 = mul_lazy_dev(q.x, p.zz);
  const Fq S1 = mul_lazy_dev(p.y, q.zzz);
  const Fq S2 = mul_lazy_dev(q.y, p.zzz);
  const Fq P = sub2_dev(U2, U1);
  const Fq R = sub2_dev(S2, S1);
  if (fq_zero_lazy(P)) {
    if (fq_zero_lazy(R)) return xyzz_dbl(xyzz_canon(p));
    return G1Xyzz::inf();
  }
  const Fq PP = sqr_lazy_dev(P);
  const Fq PPP = mul_lazy_dev(P, PP);
  const Fq Q = mul_lazy_dev(U1, PP);
  G1Xyzz r;
  r.x = sub2_dev(sub2_dev(sqr_lazy_dev(R), PPP), add2_dev(Q, Q));
  r.y = mul2_lazy_dev(R, sub2_dev(Q, r.x), S1, const_minus_dev<FqCfg, true>(PPP));  // one reduction
  r.zz = mul_lazy_dev(mul_lazy_dev(p.zz, q.zz), PP);
  r.zzz = mul_lazy_dev(mul_lazy_dev(p.zzz, q.zzz), PPP);
  return r;
}
#endif

// add-2008-s: XYZZ + XYZZ
TNS_HD G1Xyzz xyzz_add(const G1Xyzz &p, const G1Xyzz &q) {
  if (q.is_inf()) return p;
  if (p.is_inf()) return q;
  Fq U1 = mul(p.x, q.zz);
  Fq U2 = mul(q.x, p.zz);
  Fq S1 = mul(p.y, q.zzz);
  Fq S2 = mul(q.y, p.zzz);
  Fq P = sub(U2, U1);
  Fq R = sub(S2, S1);
  if (P.is_zero()) {
    if (R.is_zero()) return xyzz_dbl(p);
    return G1Xyzz::inf();
  }
  Fq PP = sqr(P);
  Fq PPP = mul(P, PP);
  Fq Q = mul(U1, PP);
  G1Xyzz r;
  r.x = sub(sub(sqr(R), PPP), dbl(Q));
  r.y = sub(mul(R, sub(Q, r.x)), mul(S1, PPP));
  r.zz = mul(mul(p.zz, q.zz), PP);
  r.zzz = mul(mul(p.zzz, q.zzz), PPP);
  return r;
}

TNS_HD G1Xyzz xyzz_from_affine(const G1Affine &a) {
  if (a.is_inf()) return G1Xyzz::inf();
  G1Xyzz r;
  r.x = a.x;
  r.y = a.y;
  r.zz = Fq::one();
  r.zzz = Fq::one();
  return r;
}

// k * p for a small non-negative integer k (double-and-add)
TNS_HD G1Xyzz xyzz_mul_small(const G1Xyzz &p, u64 k) {
  G1Xyzz acc = G1Xyzz::inf();
  for (int i = 63; i >= 0; i--) {
    acc = xyzz_dbl(acc);
    if ((k >> i) & 1) acc = xyzz_add(acc, p);
  }
  return acc;
}

// XYZZ -> affine (one field inversion)
// p with 1/ZZZ already known
TNS_HD G1Affine xyzz_to_affine_izzz(const G1Xyzz &p, const Fq &izzz) {
  G1Affine r;
  Fq iz = mul(izzz, p.zz);      // ZZ/ZZZ = 1/z  (z = ZZZ/ZZ)
  Fq izz = sqr(iz);             // 1/ZZ
  r.x = mul(p.x, izz);
  r.y = mul(p.y, izzz);
  return r;
}

TNS_HD G1Affine xyzz_to_affine(const G1Xyzz &p) {
  if (p.is_inf()) {
    G1Affine r;
    r.x = Fq::zero();
    r.y = Fq::zero();
    return r;
  }
  return xyzz_to_affine_izzz(p, inv(p.zzz));
}

// two points with ONE field inversion (Montgomery's trick): the host converts a proof's two
// commitments / two opening proofs back to back on the critical path (~19 us an inversion)
TNS_HD void xyzz_to_affine2(const G1Xyzz &p, const G1Xyzz &q, G1Affine &a, G1Affine &b) {
  if (p.is_inf() || q.is_inf()) {
    a = xyzz_to_affine(p);
    b = xyzz_to_affine(q);
    return;
  }
  const Fq it = inv(mul(p.zzz, q.zzz));
  a = xyzz_to_affine_izzz(p, mul(it, q.zzz));
  b = xyzz_to_affine_izzz(q, mul(it, p.zzz));
}

// affine -> arkworks G1Projective (Jacobian, Z = 1; identity = (1, 1, 0))
TNS_HD G1Jac affine_to_jac(const G1Affine &a) {
  G1Jac j;
  if (a.is_inf()) {
    j.x = Fq::one();
    j.y = Fq::one();
    j.z = Fq::zero();
  } else {
    j.x = a.x;
    j.y = a.y;
    j.z = Fq::one();
  }
  return j;
}

TNS_HD bool g1_on_curve(const G1Affine &a) {
  if (a.is_inf()) return true;
  Fq y2 = sqr(a.y);
  Fq x3 = mul(sqr(a.x), a.x);
  Fq three = from_u64<FqCfg>(3);
  return y2 == add(x3, three);
}

}  // namespace tns
