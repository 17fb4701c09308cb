// hostfield.hpp -- BN254 prime-field arithmetic for the host side of the verifier.
//
// The device field (bn254.hpp) works on 8 x u32 limbs because that is what the gfx950 VALU
// multiplies; on the host the natural word is 64 bits with a 128-bit product, so the pairing
// and the verifier's scalar multiplications use this 4 x u64 CIOS Montgomery form instead.
// Both forms use R = 2^256, so a value converts between them by reinterpreting its limbs.
#pragma once

#include <cstring>

#include "bn254.hpp"

namespace tns {

template <class C>
struct HCfg {
  static constexpr u64 m(int i) { return (u64)C::M[2 * i] | ((u64)C::M[2 * i + 1] << 32); }
  static constexpr u64 M[4] = {m(0), m(1), m(2), m(3)};
  static constexpr u64 inv() {  // -M^{-1} mod 2^64 (Newton)
    u64 x = 1;
    for (int i = 0; i < 7; i++) x *= 2 - M[0] * x;
    return (u64)0 - x;
  }
  static constexpr u64 INV = inv();
};

template <class C>
struct Hf {
  u64 l[4];

  static Hf zero() { return Hf{{0, 0, 0, 0}}; }
  static Hf one() { return of(Fp<C>::one()); }
  static Hf of(const Fp<C> &a) {
    Hf r;
    std::memcpy(r.l, a.v, 32);
    return r;
  }
  Fp<C> fp() const {
    Fp<C> r;
    std::memcpy(r.v, l, 32);
    return r;
  }
  bool is_zero() const { return (l[0] | l[1] | l[2] | l[3]) == 0; }
  bool operator==(const Hf &o) const {
    return ((l[0] ^ o.l[0]) | (l[1] ^ o.l[1]) | (l[2] ^ o.l[2]) | (l[3] ^ o.l[3])) == 0;
  }
  bool operator!=(const Hf &o) const { return !(*this == o); }
};

typedef unsigned __int128 u128;

// result = t - M if t >= M (t < 2M), branch-free
template <class C>
inline void h_reduce_once(u64 t[4]) {
  const u64 *M = HCfg<C>::M;
  u64 d[4], b = 0;
  for (int i = 0; i < 4; i++) {
    const u128 x = (u128)t[i] - M[i] - b;
    d[i] = (u64)x;
    b = (u64)(x >> 64) & 1;
  }
  const u64 keep = (u64)0 - b;  // all ones when t < M
  for (int i = 0; i < 4; i++) t[i] = (t[i] & keep) | (d[i] & ~keep);
}

template <class C>
inline Hf<C> operator+(const Hf<C> &a, const Hf<C> &b) {
  Hf<C> r;
  u64 c = 0;
  for (int i = 0; i < 4; i++) {
    const u128 s = (u128)a.l[i] + b.l[i] + c;
    r.l[i] = (u64)s;
    c = (u64)(s >> 64);
  }
  (void)c;  // a + b < 2M < 2^256
  h_reduce_once<C>(r.l);
  return r;
}

template <class C>
inline Hf<C> operator-(const Hf<C> &a, const Hf<C> &b) {
  Hf<C> r;
  u64 br = 0;
  for (int i = 0; i < 4; i++) {
    const u128 d = (u128)a.l[i] - b.l[i] - br;
    r.l[i] = (u64)d;
    br = (u64)(d >> 64) & 1;
  }
  const u64 mask = (u64)0 - br;  // add M back on borrow
  u64 c = 0;
  for (int i = 0; i < 4; i++) {
    const u128 s = (u128)r.l[i] + (HCfg<C>::M[i] & mask) + c;
    r.l[i] = (u64)s;
    c = (u64)(s >> 64);
  }
  return r;
}

template <class C>
inline Hf<C> operator-(const Hf<C> &a) {
  return a.is_zero() ? a : Hf<C>::zero() - a;
}

// Montgomery product a * b / 2^256 mod M: CIOS without the extra carry words, valid because
// the top limb of both moduli is below 2^63 - 1 (the partial sums stay below 2M < 2^256)
template <class C>
inline Hf<C> operator*(const Hf<C> &a, const Hf<C> &b) {
  const u64 *M = HCfg<C>::M;
  static_assert(HCfg<C>::M[3] < 0x7fffffffffffffffULL, "no-carry CIOS needs a spare top bit");
  u64 t[4] = {0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    u128 s = (u128)a.l[0] * b.l[i] + t[0];
    u64 A = (u64)(s >> 64);
    const u64 t0 = (u64)s;
    const u64 m = t0 * HCfg<C>::INV;
    s = (u128)m * M[0] + t0;
    u64 Cc = (u64)(s >> 64);
    for (int j = 1; j < 4; j++) {
      s = (u128)a.l[j] * b.l[i] + t[j] + A;
      A = (u64)(s >> 64);
      s = (u128)m * M[j] + (u64)s + Cc;
      Cc = (u64)(s >> 64);
      t[j - 1] = (u64)s;
    }
    t[3] = Cc + A;
  }
  Hf<C> r;
  for (int i = 0; i < 4; i++) r.l[i] = t[i];
  h_reduce_once<C>(r.l);
  return r;
}

template <class C>
inline Hf<C> h_dbl(const Hf<C> &a) {
  return a + a;
}

// a^e, e little-endian 64-bit limbs
template <class C>
inline Hf<C> h_pow(const Hf<C> &a, const u64 *e, int limbs) {
  Hf<C> r = Hf<C>::one();
  for (int i = limbs * 64 - 1; i >= 0; i--) {
    r = r * r;
    if ((e[i / 64] >> (i % 64)) & 1) r = r * a;
  }
  return r;
}

// a^{-1} = a^(M - 2) (0 -> 0)
template <class C>
inline Hf<C> h_inv(const Hf<C> &a) {
  u64 e[4];
  for (int i = 0; i < 4; i++) e[i] = HCfg<C>::M[i];
  e[0] -= 2;  // M is odd and > 2: no borrow
  return h_pow(a, e, 4);
}

typedef Hf<FqCfg> HFq;
typedef Hf<FrCfg> HFr;

}  // namespace tns
