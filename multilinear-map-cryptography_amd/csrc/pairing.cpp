// pairing.cpp -- BN254 optimal ate pairing and the KZG / Twist / Shout verifiers (host).
//
// the verifier closes the prove -> verify loop every reference
// integration test runs (`Twist::verify`, `Shout::verify`, src/twist.rs:255-304,
// src/shout.rs:225-274; `KZGCommitment::verify` / `batch_verify`, src/commitments.rs:201-301,
// arkworks `Bn254::pairing`).  It is O(1) pairings per proof -- host code, not a GPU kernel.
//
// Tower: Fq2 = Fq[u]/(u^2 + 1), Fq6 = Fq2[v]/(v^3 - xi), Fq12 = Fq6[w]/(w^2 - v), xi = 9 + u.
// G2 is the D-type sextic twist E': y^2 = x^3 + 3/xi; psi(x, y) = (x w^2, y w^3) maps it into
// E(Fq12), where the Miller loop runs with plain affine chord/tangent lines (vertical lines
// lie in Fq6 and vanish under the final exponentiation).  Optimal ate:
//   f = f_{6x+2,Q}(P) * l_{T,pi(Q)}(P) * l_{T+pi(Q),-pi^2(Q)}(P),  T = [6x+2]Q,
//   e(P, Q) = f^((p^12 - 1) / r),  x = 4965661367192848881.
// The reduced pairing is unique, so every correct implementation (arkworks' included) gives
// the same value; the verifiers only compare pairings.
#include <cstring>
#include <string>
#include <vector>

#include "common.hpp"
#include "hostfield.hpp"

namespace tns {

namespace {

typedef HFq F;

// ---------------------------------------------------------------- Fq2
struct Fq2 {
  F c0, c1;
};
inline Fq2 f2_zero() { return Fq2{F::zero(), F::zero()}; }
inline Fq2 f2_one() { return Fq2{F::one(), F::zero()}; }
inline bool f2_eq(const Fq2 &a, const Fq2 &b) { return a.c0 == b.c0 && a.c1 == b.c1; }
inline bool f2_is_zero(const Fq2 &a) { return a.c0.is_zero() && a.c1.is_zero(); }
inline Fq2 f2_add(const Fq2 &a, const Fq2 &b) { return Fq2{a.c0 + b.c0, a.c1 + b.c1}; }
inline Fq2 f2_sub(const Fq2 &a, const Fq2 &b) { return Fq2{a.c0 - b.c0, a.c1 - b.c1}; }
inline Fq2 f2_neg(const Fq2 &a) { return Fq2{-a.c0, -a.c1}; }
inline Fq2 f2_dbl(const Fq2 &a) { return f2_add(a, a); }
inline Fq2 f2_conj(const Fq2 &a) { return Fq2{a.c0, -a.c1}; }  // a^p
inline Fq2 f2_mul(const Fq2 &a, const Fq2 &b) {  // Karatsuba, u^2 = -1
  const F t0 = a.c0 * b.c0, t1 = a.c1 * b.c1;
  const F t2 = (a.c0 + a.c1) * (b.c0 + b.c1);
  return Fq2{t0 - t1, t2 - t0 - t1};
}
inline Fq2 f2_sqr(const Fq2 &a) {  // (a0 + a1)(a0 - a1) + 2 a0 a1 u
  const F t = a.c0 * a.c1;
  return Fq2{(a.c0 + a.c1) * (a.c0 - a.c1), t + t};
}
inline Fq2 f2_scale(const Fq2 &a, const F &k) { return Fq2{a.c0 * k, a.c1 * k}; }
inline Fq2 f2_inv(const Fq2 &a) {
  const F n = h_inv(a.c0 * a.c0 + a.c1 * a.c1);
  return Fq2{a.c0 * n, -(a.c1 * n)};
}
// multiplication by xi = 9 + u
inline Fq2 f2_mul_xi(const Fq2 &a) {
  const F a2 = a.c0 + a.c0, a4 = a2 + a2, a8 = a4 + a4;
  const F b2 = a.c1 + a.c1, b4 = b2 + b2, b8 = b4 + b4;
  return Fq2{a8 + a.c0 - a.c1, b8 + a.c1 + a.c0};
}
Fq2 f2_pow(const Fq2 &a, const u64 *e, int limbs) {
  Fq2 r = f2_one();
  for (int i = limbs * 64 - 1; i >= 0; i--) {
    r = f2_sqr(r);
    if ((e[i / 64] >> (i % 64)) & 1) r = f2_mul(r, a);
  }
  return r;
}

// ---------------------------------------------------------------- Fq6
struct Fq6 {
  Fq2 c0, c1, c2;
};
inline Fq6 f6_zero() { return Fq6{f2_zero(), f2_zero(), f2_zero()}; }
inline Fq6 f6_one() { return Fq6{f2_one(), f2_zero(), f2_zero()}; }
inline bool f6_eq(const Fq6 &a, const Fq6 &b) { return f2_eq(a.c0, b.c0) && f2_eq(a.c1, b.c1) && f2_eq(a.c2, b.c2); }
inline Fq6 f6_add(const Fq6 &a, const Fq6 &b) { return Fq6{f2_add(a.c0, b.c0), f2_add(a.c1, b.c1), f2_add(a.c2, b.c2)}; }
inline Fq6 f6_sub(const Fq6 &a, const Fq6 &b) { return Fq6{f2_sub(a.c0, b.c0), f2_sub(a.c1, b.c1), f2_sub(a.c2, b.c2)}; }
inline Fq6 f6_neg(const Fq6 &a) { return Fq6{f2_neg(a.c0), f2_neg(a.c1), f2_neg(a.c2)}; }
inline Fq6 f6_mul(const Fq6 &a, const Fq6 &b) {  // Karatsuba over v^3 = xi: 6 Fq2 products
  const Fq2 v0 = f2_mul(a.c0, b.c0), v1 = f2_mul(a.c1, b.c1), v2 = f2_mul(a.c2, b.c2);
  const Fq2 c0 = f2_add(v0, f2_mul_xi(f2_sub(f2_sub(f2_mul(f2_add(a.c1, a.c2), f2_add(b.c1, b.c2)), v1), v2)));
  const Fq2 c1 = f2_add(f2_sub(f2_sub(f2_mul(f2_add(a.c0, a.c1), f2_add(b.c0, b.c1)), v0), v1), f2_mul_xi(v2));
  const Fq2 c2 = f2_add(f2_sub(f2_sub(f2_mul(f2_add(a.c0, a.c2), f2_add(b.c0, b.c2)), v0), v2), v1);
  return Fq6{c0, c1, c2};
}
// multiplication by v
inline Fq6 f6_mul_v(const Fq6 &a) { return Fq6{f2_mul_xi(a.c2), a.c0, a.c1}; }
// a * (b + c v)
inline Fq6 f6_mul_01(const Fq6 &a, const Fq2 &b, const Fq2 &c) {
  return Fq6{f2_add(f2_mul(a.c0, b), f2_mul_xi(f2_mul(a.c2, c))), f2_add(f2_mul(a.c0, c), f2_mul(a.c1, b)),
             f2_add(f2_mul(a.c1, c), f2_mul(a.c2, b))};
}
inline Fq6 f6_scale(const Fq6 &a, const F &k) { return Fq6{f2_scale(a.c0, k), f2_scale(a.c1, k), f2_scale(a.c2, k)}; }
inline Fq6 f6_inv(const Fq6 &a) {
  const Fq2 t0 = f2_sub(f2_sqr(a.c0), f2_mul_xi(f2_mul(a.c1, a.c2)));
  const Fq2 t1 = f2_sub(f2_mul_xi(f2_sqr(a.c2)), f2_mul(a.c0, a.c1));
  const Fq2 t2 = f2_sub(f2_sqr(a.c1), f2_mul(a.c0, a.c2));
  const Fq2 d = f2_add(f2_mul(a.c0, t0), f2_mul_xi(f2_add(f2_mul(a.c2, t1), f2_mul(a.c1, t2))));
  const Fq2 di = f2_inv(d);
  return Fq6{f2_mul(t0, di), f2_mul(t1, di), f2_mul(t2, di)};
}

// ---------------------------------------------------------------- Fq12
struct Fq12 {
  Fq6 c0, c1;
};
inline Fq12 f12_one() { return Fq12{f6_one(), f6_zero()}; }
inline bool f12_eq(const Fq12 &a, const Fq12 &b) { return f6_eq(a.c0, b.c0) && f6_eq(a.c1, b.c1); }
inline Fq12 f12_mul(const Fq12 &a, const Fq12 &b) {
  const Fq6 t0 = f6_mul(a.c0, b.c0), t1 = f6_mul(a.c1, b.c1);
  const Fq6 t2 = f6_mul(f6_add(a.c0, a.c1), f6_add(b.c0, b.c1));
  return Fq12{f6_add(t0, f6_mul_v(t1)), f6_sub(f6_sub(t2, t0), t1)};
}
inline Fq12 f12_sqr(const Fq12 &a) {  // complex squaring: 2 Fq6 products
  const Fq6 t = f6_mul(a.c0, a.c1);
  const Fq6 s = f6_mul(f6_add(a.c0, a.c1), f6_add(a.c0, f6_mul_v(a.c1)));
  return Fq12{f6_sub(f6_sub(s, t), f6_mul_v(t)), f6_add(t, t)};
}
inline Fq12 f12_conj(const Fq12 &a) { return Fq12{a.c0, f6_neg(a.c1)}; }  // a^(p^6)
inline Fq12 f12_inv(const Fq12 &a) {
  const Fq6 d = f6_inv(f6_sub(f6_mul(a.c0, a.c0), f6_mul_v(f6_mul(a.c1, a.c1))));
  return Fq12{f6_mul(a.c0, d), f6_neg(f6_mul(a.c1, d))};
}
// f * l for a line l = a + (b + c v) w (a in Fq): the shape every Miller-loop line has
inline Fq12 f12_mul_line(const Fq12 &f, const F &a, const Fq2 &b, const Fq2 &c) {
  return Fq12{f6_add(f6_scale(f.c0, a), f6_mul_v(f6_mul_01(f.c1, b, c))),
              f6_add(f6_mul_01(f.c0, b, c), f6_scale(f.c1, a))};
}
inline bool f12_is_one(const Fq12 &a) { return f12_eq(a, f12_one()); }

// Frobenius: in the basis w^k (v = w^2), a = sum a_k w^k with a_k in Fq2 and
// (a_k w^k)^p = conj(a_k) w^k gamma^k, gamma = w^(p-1) = xi^((p-1)/6)   (p = 1 mod 6)
struct Frob {
  Fq2 g[6];
  Frob() {
    u64 e[4];
    for (int i = 0; i < 4; i++) e[i] = HCfg<FqCfg>::M[i];
    e[0] -= 1;
    u128 rem = 0;  // (p - 1) / 6, long division from the top limb
    for (int i = 3; i >= 0; i--) {
      const u128 cur = (rem << 64) | e[i];
      e[i] = (u64)(cur / 6);
      rem = cur % 6;
    }
    const Fq2 gam = f2_pow(f2_mul_xi(f2_one()), e, 4);
    g[0] = f2_one();
    for (int k = 1; k < 6; k++) g[k] = f2_mul(g[k - 1], gam);
  }
};
const Frob &frob_consts() {
  static const Frob f;
  return f;
}
Fq12 f12_frob(const Fq12 &a) {  // a^p
  const Fq2 *g = frob_consts().g;
  return Fq12{Fq6{f2_conj(a.c0.c0), f2_mul(f2_conj(a.c0.c1), g[2]), f2_mul(f2_conj(a.c0.c2), g[4])},
              Fq6{f2_mul(f2_conj(a.c1.c0), g[1]), f2_mul(f2_conj(a.c1.c1), g[3]), f2_mul(f2_conj(a.c1.c2), g[5])}};
}

const uint64_t ATE_LOOP = 0x9d797039be763ba8ULL;  // 6x + 2 = 2^64 + this (65 bits)

// Squaring in the cyclotomic subgroup (Granger-Scott): view a as three Fq4 = Fq2[y]/(y^2 - xi)
// elements, y = w^3:  A = c0.c0 + c1.c1 y,  B = c1.c0 + c0.c2 y,  C = c0.c1 + c1.c2 y; then
// A' = 3A^2 - 2 conj(A),  B' = 3 y C^2 + 2 conj(B),  C' = 3B^2 - 2 conj(C)   (valid after the easy part)
inline void fq4_sqr(const Fq2 &a, const Fq2 &b, Fq2 &t0, Fq2 &t1) {  // (a + b y)^2 = t0 + t1 y
  const Fq2 ab = f2_mul(a, b);
  t0 = f2_sub(f2_sub(f2_mul(f2_add(a, b), f2_add(a, f2_mul_xi(b))), ab), f2_mul_xi(ab));
  t1 = f2_dbl(ab);
}
inline Fq2 three_minus_two(const Fq2 &t, const Fq2 &z) { return f2_add(f2_dbl(f2_sub(t, z)), t); }  // 3t - 2z
inline Fq2 three_plus_two(const Fq2 &t, const Fq2 &z) { return f2_add(f2_dbl(f2_add(t, z)), t); }   // 3t + 2z
Fq12 cyclo_sqr(const Fq12 &a) {
  Fq2 t0, t1, t2, t3, t4, t5;
  fq4_sqr(a.c0.c0, a.c1.c1, t0, t1);  // A^2
  fq4_sqr(a.c1.c0, a.c0.c2, t2, t3);  // B^2
  fq4_sqr(a.c0.c1, a.c1.c2, t4, t5);  // C^2
  Fq12 r;
  r.c0.c0 = three_minus_two(t0, a.c0.c0);
  r.c1.c1 = three_plus_two(t1, a.c1.c1);
  r.c1.c0 = three_plus_two(f2_mul_xi(t5), a.c1.c0);
  r.c0.c2 = three_minus_two(t4, a.c0.c2);
  r.c0.c1 = three_minus_two(t2, a.c0.c1);
  r.c1.c2 = three_plus_two(t3, a.c1.c2);
  return r;
}
// a^X for the BN parameter X = 4965661367192848881 (a in the cyclotomic subgroup)
const uint64_t BN_X = 0x44e992b44a6909f1ULL;
Fq12 cyclo_exp_x(const Fq12 &a) {
  Fq12 r = a;
  for (int i = 61; i >= 0; i--) {
    r = cyclo_sqr(r);
    if ((BN_X >> i) & 1) r = f12_mul(r, a);
  }
  return r;
}
Fq12 cyclo_pow_small(const Fq12 &a, unsigned e) {  // e >= 1
  int top = 31 - __builtin_clz(e);
  Fq12 r = a;
  for (int i = top - 1; i >= 0; i--) {
    r = cyclo_sqr(r);
    if ((e >> i) & 1) r = f12_mul(r, a);
  }
  return r;
}

Fq12 final_exp(const Fq12 &f) {
  // easy part: f^((p^6 - 1)(p^2 + 1))
  Fq12 t = f12_mul(f12_conj(f), f12_inv(f));
  t = f12_mul(f12_frob(f12_frob(t)), t);
  // hard part: ^((p^4 - p^2 + 1) / r) = l0 + l1 p + l2 p^2 + p^3 exactly, with
  //   l0 = -36X^3 - 30X^2 - 18X - 2,  l1 = -36X^3 - 18X^2 - 12X + 1,  l2 = 6X^2 + 1
  // (inversion is conjugation in the cyclotomic subgroup)
  const Fq12 a = cyclo_exp_x(t), b = cyclo_exp_x(a), c = cyclo_exp_x(b);  // t^X, t^X^2, t^X^3
  const Fq12 c36 = cyclo_pow_small(c, 36);
  const Fq12 f0 = f12_conj(f12_mul(f12_mul(c36, cyclo_pow_small(b, 30)), f12_mul(cyclo_pow_small(a, 18), cyclo_sqr(t))));
  const Fq12 f1 = f12_mul(f12_conj(f12_mul(f12_mul(c36, cyclo_pow_small(b, 18)), cyclo_pow_small(a, 12))), t);
  const Fq12 f2 = f12_mul(cyclo_pow_small(b, 6), t);
  const Fq12 r = f12_mul(f12_mul(f0, f12_frob(f1)), f12_mul(f12_frob(f12_frob(f2)), f12_frob(f12_frob(f12_frob(t)))));
  return r;
}

// ---------------------------------------------------------------- Miller loop on the twist
// T on E'(Fq2): y^2 = x^3 + b', b' = 3/xi, in homogeneous projective coordinates (X : Y : Z).
// psi(x, y) = (x w^2, y w^3) puts E' into E(Fq12) and turns a slope lambda' into lambda' w, so the
// line through psi(T) and psi(S) evaluated at P = (xP, yP) is
//     yP - lambda' xP w + (lambda' xS - yS) w^3.
// Lines are kept up to a factor in Fq2 (killed by the final exponentiation), which removes every
// inversion:  l = A yP + B xP w + C w^3  with A, B, C in Fq2.
struct TwistPt {
  Fq2 x, y;
};
struct TwistProj {
  Fq2 X, Y, Z;
};
struct Line {
  Fq2 a, b, c;  // l = a + b w + c w^3 (yP, xP already folded in)
};

const Fq2 &twist_b() {
  static const Fq2 b = f2_mul(Fq2{F::of(from_u64<FqCfg>(3)), F::zero()}, f2_inv(f2_mul_xi(f2_one())));
  return b;
}

// tangent at T: lambda' = 3x^2 / 2y = 3X^2 / 2YZ.  Times 2YZ, and with X^3 = Y^2 Z - b'Z^3:
//   l ~ 2YZ yP - 3X^2 xP w + (Y^2 - 3b'Z^2) w^3
// 2T, scaled by 4 to avoid halves (e = 3b'Z^2):
//   (2XY (Y^2 - 3e) : (Y^2 + 3e)^2 - 12 e^2 : 8 Y^3 Z)
inline Line dbl_step(TwistProj &T, const F &xP, const F &yP) {
  const Fq2 &bt = twist_b();
  const Fq2 X2 = f2_sqr(T.X), Y2 = f2_sqr(T.Y), Z2 = f2_sqr(T.Z);
  const Fq2 e = f2_mul(f2_add(f2_dbl(bt), bt), Z2);                   // 3b'Z^2
  const Fq2 e3 = f2_add(f2_dbl(e), e);                                 // 9b'Z^2
  const Fq2 YZ2 = f2_sub(f2_sub(f2_sqr(f2_add(T.Y, T.Z)), Y2), Z2);  // 2YZ
  const Line l{f2_scale(YZ2, yP), f2_neg(f2_scale(f2_add(f2_dbl(X2), X2), xP)), f2_sub(Y2, e)};
  const Fq2 ee = f2_sqr(e);
  T.X = f2_dbl(f2_mul(f2_mul(T.X, T.Y), f2_sub(Y2, e3)));
  T.Y = f2_sub(f2_sqr(f2_add(Y2, e3)), f2_dbl(f2_dbl(f2_add(f2_dbl(ee), ee))));
  T.Z = f2_dbl(f2_dbl(f2_mul(Y2, YZ2)));
  return l;
}

// chord through T and Q (affine): theta = Y - yQ Z, mu = X - xQ Z, lambda' = theta / mu;
//   l ~ mu yP - theta xP w + (theta xQ - mu yQ) w^3
// T + Q: c = theta^2, d = mu^2, e = mu^3, f = Z c, g = X d, h = e + f - 2g:
//   (mu h : theta (g - h) - e Y : Z e)
inline Line add_step(TwistProj &T, const TwistPt &Q, const F &xP, const F &yP) {
  const Fq2 theta = f2_sub(T.Y, f2_mul(Q.y, T.Z)), mu = f2_sub(T.X, f2_mul(Q.x, T.Z));
  const Line l{f2_scale(mu, yP), f2_neg(f2_scale(theta, xP)), f2_sub(f2_mul(theta, Q.x), f2_mul(mu, Q.y))};
  const Fq2 c = f2_sqr(theta), d = f2_sqr(mu);
  const Fq2 e = f2_mul(mu, d), f = f2_mul(T.Z, c), g = f2_mul(T.X, d);
  const Fq2 h = f2_sub(f2_add(e, f), f2_dbl(g));
  T.X = f2_mul(mu, h);
  T.Y = f2_sub(f2_mul(theta, f2_sub(g, h)), f2_mul(e, T.Y));
  T.Z = f2_mul(T.Z, e);
  return l;
}

// f * (a + b w + c w^3) = f * (a + (b + c v) w)
inline Fq12 f12_mul_line(const Fq12 &f, const Line &l) {
  const Fq6 f0a{f2_mul(f.c0.c0, l.a), f2_mul(f.c0.c1, l.a), f2_mul(f.c0.c2, l.a)};
  const Fq6 f1a{f2_mul(f.c1.c0, l.a), f2_mul(f.c1.c1, l.a), f2_mul(f.c1.c2, l.a)};
  return Fq12{f6_add(f0a, f6_mul_v(f6_mul_01(f.c1, l.b, l.c))), f6_add(f6_mul_01(f.c0, l.b, l.c), f1a)};
}

struct PairIn {
  F xP, yP;
  TwistPt q;
};

// prod_k f_{6x+2,Q_k}(P_k) * lines through pi(Q_k), -pi^2(Q_k): one shared accumulator
Fq12 miller_multi(const std::vector<PairIn> &in) {
  Fq12 f = f12_one();
  std::vector<TwistProj> T(in.size());
  for (size_t k = 0; k < in.size(); k++) T[k] = TwistProj{in[k].q.x, in[k].q.y, f2_one()};
  for (int i = 63; i >= 0; i--) {
    f = f12_sqr(f);
    for (size_t k = 0; k < in.size(); k++) f = f12_mul_line(f, dbl_step(T[k], in[k].xP, in[k].yP));
    if ((ATE_LOOP >> i) & 1)
      for (size_t k = 0; k < in.size(); k++) f = f12_mul_line(f, add_step(T[k], in[k].q, in[k].xP, in[k].yP));
  }
  const Fq2 *g = frob_consts().g;
  for (size_t k = 0; k < in.size(); k++) {
    const TwistPt &q = in[k].q;
    const TwistPt q1{f2_mul(f2_conj(q.x), g[2]), f2_mul(f2_conj(q.y), g[3])};            // pi(Q)
    const TwistPt q2{f2_mul(f2_conj(q1.x), g[2]), f2_neg(f2_mul(f2_conj(q1.y), g[3]))};  // -pi^2(Q)
    f = f12_mul_line(f, add_step(T[k], q1, in[k].xP, in[k].yP));
    f = f12_mul_line(f, add_step(T[k], q2, in[k].xP, in[k].yP));
  }
  return f;
}

}  // namespace

// ---------------------------------------------------------------- public (tns::)
G2Affine g2_generator() {
  static const uint64_t G[16] = {
      0x46debd5cd992f6edULL, 0x674322d4f75edaddULL, 0x426a00665e5c4479ULL, 0x1800deef121f1e76ULL,   // x.c0
      0x97e485b7aef312c2ULL, 0xf1aa493335a9e712ULL, 0x7260bfb731fb5d25ULL, 0x198e9393920d483aULL,   // x.c1
      0x4ce6cc0166fa7daaULL, 0xe3d1e7690c43d37bULL, 0x4aab71808dcb408fULL, 0x12c85ea5db8c6debULL,   // y.c0
      0x55acdadcd122975bULL, 0xbc4b313370b38ef3ULL, 0xec9e99ad690c3395ULL, 0x090689d0585ff075ULL};  // y.c1
  G2Affine g;
  Fq *c[4] = {&g.x0, &g.x1, &g.y0, &g.y1};
  for (int k = 0; k < 4; k++) {
    Fq v;
    std::memcpy(&v, G + 4 * k, 32);
    *c[k] = to_mont(v);
  }
  g.inf = false;
  return g;
}

namespace {
Fq2 gx(const G2Affine &a) { return Fq2{F::of(a.x0), F::of(a.x1)}; }
Fq2 gy(const G2Affine &a) { return Fq2{F::of(a.y0), F::of(a.y1)}; }
G2Affine mk(const Fq2 &x, const Fq2 &y) {
  G2Affine r;
  r.x0 = x.c0.fp();
  r.x1 = x.c1.fp();
  r.y0 = y.c0.fp();
  r.y1 = y.c1.fp();
  r.inf = false;
  return r;
}
G2Affine g2_inf() {
  G2Affine r;
  r.x0 = r.x1 = r.y0 = r.y1 = Fq::zero();
  r.inf = true;
  return r;
}

// Jacobian (X, Y, Z) on E': y^2 = x^3 + b' (a = 0); Z = 0 is the identity
struct G2J {
  Fq2 X, Y, Z;
};
G2J j_dbl(const G2J &p) {  // dbl-2009-l
  if (f2_is_zero(p.Z)) return p;
  const Fq2 A = f2_sqr(p.X), B = f2_sqr(p.Y), C = f2_sqr(B);
  const Fq2 D = f2_dbl(f2_sub(f2_sub(f2_sqr(f2_add(p.X, B)), A), C));
  const Fq2 E = f2_add(f2_dbl(A), A), Fv = f2_sqr(E);
  const Fq2 X3 = f2_sub(Fv, f2_dbl(D));
  const Fq2 C8 = f2_dbl(f2_dbl(f2_dbl(C)));
  return G2J{X3, f2_sub(f2_mul(E, f2_sub(D, X3)), C8), f2_dbl(f2_mul(p.Y, p.Z))};
}
G2J j_add_affine(const G2J &p, const TwistPt &q) {  // madd-2007-bl, with the doubling case
  if (f2_is_zero(p.Z)) return G2J{q.x, q.y, f2_one()};
  const Fq2 Z1Z1 = f2_sqr(p.Z);
  const Fq2 U2 = f2_mul(q.x, Z1Z1), S2 = f2_mul(f2_mul(q.y, p.Z), Z1Z1);
  const Fq2 H = f2_sub(U2, p.X), r = f2_dbl(f2_sub(S2, p.Y));
  if (f2_is_zero(H)) {
    if (f2_is_zero(r)) return j_dbl(p);
    return G2J{f2_one(), f2_one(), f2_zero()};
  }
  const Fq2 HH = f2_sqr(H), I = f2_dbl(f2_dbl(HH)), J = f2_mul(H, I), V = f2_mul(p.X, I);
  const Fq2 X3 = f2_sub(f2_sub(f2_sqr(r), J), f2_dbl(V));
  const Fq2 Y3 = f2_sub(f2_mul(r, f2_sub(V, X3)), f2_dbl(f2_mul(p.Y, J)));
  const Fq2 Z3 = f2_sub(f2_sub(f2_sqr(f2_add(p.Z, H)), Z1Z1), HH);
  return G2J{X3, Y3, Z3};
}
}  // namespace

G2Affine g2_add(const G2Affine &a, const G2Affine &b) {
  if (a.inf) return b;
  if (b.inf) return a;
  const Fq2 ax = gx(a), ay = gy(a), bx = gx(b), by = gy(b);
  Fq2 lam;
  if (f2_eq(ax, bx)) {
    if (!f2_eq(ay, by) || f2_is_zero(ay)) return g2_inf();
    const Fq2 x2 = f2_sqr(ax);
    lam = f2_mul(f2_add(f2_dbl(x2), x2), f2_inv(f2_dbl(ay)));
  } else {
    lam = f2_mul(f2_sub(by, ay), f2_inv(f2_sub(bx, ax)));
  }
  const Fq2 x3 = f2_sub(f2_sub(f2_sqr(lam), ax), bx);
  const Fq2 y3 = f2_sub(f2_mul(lam, f2_sub(ax, x3)), ay);
  return mk(x3, y3);
}

G2Affine g2_neg(const G2Affine &a) {
  if (a.inf) return a;
  return mk(gx(a), f2_neg(gy(a)));
}

// k * a for a canonical scalar k (little-endian 64-bit limbs): Jacobian double-and-add,
// one inversion at the end
G2Affine g2_mul(const G2Affine &a, const uint64_t k[4]) {
  if (a.inf) return a;
  const TwistPt q{gx(a), gy(a)};
  G2J r{f2_one(), f2_one(), f2_zero()};
  for (int i = 255; i >= 0; i--) {
    r = j_dbl(r);
    if ((k[i / 64] >> (i % 64)) & 1) r = j_add_affine(r, q);
  }
  if (f2_is_zero(r.Z)) return g2_inf();
  const Fq2 zi = f2_inv(r.Z), zi2 = f2_sqr(zi);
  return mk(f2_mul(r.X, zi2), f2_mul(r.Y, f2_mul(zi2, zi)));
}

bool g2_on_curve(const G2Affine &a) {
  if (a.inf) return true;
  const Fq2 three{F::of(from_u64<FqCfg>(3)), F::zero()};
  const Fq2 b = f2_mul(three, f2_inv(f2_mul_xi(f2_one())));
  const Fq2 x = gx(a), y = gy(a);
  return f2_eq(f2_sqr(y), f2_add(f2_mul(f2_sqr(x), x), b));
}

// e(P1, Q1) == e(P2, Q2)  <=>  FE(f_{Q1}(P1) * f_{Q2}(-P2)) == 1: one shared Miller loop, one
// final exponentiation (identity inputs contribute 1)
bool pairing_eq(const G1Affine &P1, const G2Affine &Q1, const G1Affine &P2, const G2Affine &Q2) {
  std::vector<PairIn> in;
  if (!P1.is_inf() && !Q1.inf) in.push_back(PairIn{F::of(P1.x), F::of(P1.y), TwistPt{gx(Q1), gy(Q1)}});
  if (!P2.is_inf() && !Q2.inf) in.push_back(PairIn{F::of(P2.x), -F::of(P2.y), TwistPt{gx(Q2), gy(Q2)}});
  if (in.empty()) return true;
  return f12_is_one(final_exp(miller_multi(in)));
}

// e(P, Q) as 12 Fq (Montgomery), coefficient order c0.c0.c0, c0.c0.c1, c0.c1.c0, ..., c1.c2.c1
void pairing_value(const G1Affine &P, const G2Affine &Q, Fq out[12]) {
  Fq12 e = f12_one();
  if (!P.is_inf() && !Q.inf) e = final_exp(miller_multi({PairIn{F::of(P.x), F::of(P.y), TwistPt{gx(Q), gy(Q)}}}));
  const Fq6 *s[2] = {&e.c0, &e.c1};
  int k = 0;
  for (int i = 0; i < 2; i++) {
    const Fq2 *t[3] = {&s[i]->c0, &s[i]->c1, &s[i]->c2};
    for (int j = 0; j < 3; j++) {
      out[k++] = t[j]->c0.fp();
      out[k++] = t[j]->c1.fp();
    }
  }
}

}  // namespace tns
