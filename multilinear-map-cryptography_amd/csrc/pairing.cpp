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

namespace tns {

namespace {

// ---------------------------------------------------------------- Fq2
struct Fq2 {
  Fq c0, c1;
};
inline Fq2 f2(const Fq &a, const Fq &b) { return Fq2{a, b}; }
inline Fq2 f2_zero() { return Fq2{Fq::zero(), Fq::zero()}; }
inline Fq2 f2_one() { return Fq2{Fq::one(), Fq::zero()}; }
inline bool f2_eq(const Fq2 &a, const Fq2 &b) { return a.c0 == b.c0 && a.c1 == b.c1; }
inline bool f2_is_zero(const Fq2 &a) { return a.c0.is_zero() && a.c1.is_zero(); }
inline Fq2 f2_add(const Fq2 &a, const Fq2 &b) { return Fq2{add(a.c0, b.c0), add(a.c1, b.c1)}; }
inline Fq2 f2_sub(const Fq2 &a, const Fq2 &b) { return Fq2{sub(a.c0, b.c0), sub(a.c1, b.c1)}; }
inline Fq2 f2_neg(const Fq2 &a) { return Fq2{neg(a.c0), neg(a.c1)}; }
inline Fq2 f2_mul(const Fq2 &a, const Fq2 &b) {
  const Fq t0 = mul(a.c0, b.c0), t1 = mul(a.c1, b.c1);
  const Fq t2 = mul(add(a.c0, a.c1), add(b.c0, b.c1));
  return Fq2{sub(t0, t1), sub(sub(t2, t0), t1)};
}
inline Fq2 f2_sqr(const Fq2 &a) { return f2_mul(a, a); }
inline Fq2 f2_scale(const Fq2 &a, const Fq &k) { return Fq2{mul(a.c0, k), mul(a.c1, k)}; }
inline Fq2 f2_inv(const Fq2 &a) {
  const Fq n = inv(add(sqr(a.c0), sqr(a.c1)));
  return Fq2{mul(a.c0, n), neg(mul(a.c1, n))};
}
// multiplication by xi = 9 + u
inline Fq2 f2_mul_xi(const Fq2 &a) {
  const Fq nine = from_u64<FqCfg>(9);
  return Fq2{sub(mul(a.c0, nine), a.c1), add(mul(a.c1, nine), a.c0)};
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
inline Fq6 f6_mul(const Fq6 &a, const Fq6 &b) {
  // schoolbook with v^3 = xi
  const Fq2 a0b0 = f2_mul(a.c0, b.c0), a1b1 = f2_mul(a.c1, b.c1), a2b2 = f2_mul(a.c2, b.c2);
  const Fq2 c0 = f2_add(a0b0, f2_mul_xi(f2_add(f2_mul(a.c1, b.c2), f2_mul(a.c2, b.c1))));
  const Fq2 c1 = f2_add(f2_add(f2_mul(a.c0, b.c1), f2_mul(a.c1, b.c0)), f2_mul_xi(a2b2));
  const Fq2 c2 = f2_add(f2_add(f2_mul(a.c0, b.c2), f2_mul(a.c2, b.c0)), a1b1);
  return Fq6{c0, c1, c2};
}
// multiplication by v
inline Fq6 f6_mul_v(const Fq6 &a) { return Fq6{f2_mul_xi(a.c2), a.c0, a.c1}; }
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
inline Fq12 f12_add(const Fq12 &a, const Fq12 &b) { return Fq12{f6_add(a.c0, b.c0), f6_add(a.c1, b.c1)}; }
inline Fq12 f12_sub(const Fq12 &a, const Fq12 &b) { return Fq12{f6_sub(a.c0, b.c0), f6_sub(a.c1, b.c1)}; }
inline Fq12 f12_neg(const Fq12 &a) { return Fq12{f6_neg(a.c0), f6_neg(a.c1)}; }
inline Fq12 f12_mul(const Fq12 &a, const Fq12 &b) {
  const Fq6 t0 = f6_mul(a.c0, b.c0), t1 = f6_mul(a.c1, b.c1);
  const Fq6 t2 = f6_mul(f6_add(a.c0, a.c1), f6_add(b.c0, b.c1));
  return Fq12{f6_add(t0, f6_mul_v(t1)), f6_sub(f6_sub(t2, t0), t1)};
}
inline Fq12 f12_sqr(const Fq12 &a) { return f12_mul(a, a); }
inline Fq12 f12_conj(const Fq12 &a) { return Fq12{a.c0, f6_neg(a.c1)}; }  // a^(p^6)
inline Fq12 f12_inv(const Fq12 &a) {
  const Fq6 d = f6_inv(f6_sub(f6_mul(a.c0, a.c0), f6_mul_v(f6_mul(a.c1, a.c1))));
  return Fq12{f6_mul(a.c0, d), f6_neg(f6_mul(a.c1, d))};
}
// a^e, e little-endian 64-bit limbs
Fq12 f12_pow(const Fq12 &a, const uint64_t *e, int limbs) {
  Fq12 r = f12_one();
  for (int i = limbs * 64 - 1; i >= 0; i--) {
    r = f12_sqr(r);
    if ((e[i / 64] >> (i % 64)) & 1) r = f12_mul(r, a);
  }
  return r;
}
inline bool f12_is_one(const Fq12 &a) { return f12_eq(a, f12_one()); }

// the field modulus p as 64-bit limbs
void p_limbs(uint64_t out[4]) {
  for (int i = 0; i < 4; i++) out[i] = (uint64_t)FqCfg::M[2 * i] | ((uint64_t)FqCfg::M[2 * i + 1] << 32);
}
Fq12 f12_frob(const Fq12 &a) {  // a^p
  uint64_t pl[4];
  p_limbs(pl);
  return f12_pow(a, pl, 4);
}

// (p^4 - p^2 + 1) / r, little-endian
const uint64_t HARD_EXP[12] = {
    0xe81bb482ccdf42b1ULL, 0x5abf5cc4f49c36d4ULL, 0xf1154e7e1da014fdULL, 0xdcc7b44c87cdbacfULL,
    0xaaa441e3954bcf8aULL, 0x6b887d56d5095f23ULL, 0x79581e16f3fd90c6ULL, 0x3b1b1355d189227dULL,
    0x4e529a5861876f6bULL, 0x6c0eb522d5b12278ULL, 0x331ec15183177fafULL, 0x01baaa710b0759adULL};
const uint64_t ATE_LOOP = 0x9d797039be763ba8ULL;  // 6x + 2 = 2^64 + this (65 bits)

Fq12 final_exp(const Fq12 &f) {
  // easy part: f^((p^6 - 1)(p^2 + 1))
  Fq12 t = f12_mul(f12_conj(f), f12_inv(f));
  t = f12_mul(f12_frob(f12_frob(t)), t);
  // hard part: ^((p^4 - p^2 + 1) / r)
  return f12_pow(t, HARD_EXP, 12);
}

// ---------------------------------------------------------------- curve points in E(Fq12)
struct P12 {
  Fq12 x, y;
  bool inf;
};

Fq12 embed_fq(const Fq &a) {
  Fq12 r{f6_zero(), f6_zero()};
  r.c0.c0.c0 = a;
  return r;
}

// line through T and S (tangent if T == S) evaluated at P, and T + S
Fq12 line_step(P12 &T, const P12 &S, const Fq12 &xP, const Fq12 &yP, bool tangent) {
  Fq12 lam;
  if (tangent) {
    const Fq12 x2 = f12_sqr(T.x);
    lam = f12_mul(f12_add(f12_add(x2, x2), x2), f12_inv(f12_add(T.y, T.y)));
  } else {
    lam = f12_mul(f12_sub(S.y, T.y), f12_inv(f12_sub(S.x, T.x)));
  }
  const Fq12 l = f12_sub(f12_sub(yP, T.y), f12_mul(lam, f12_sub(xP, T.x)));
  const Fq12 x3 = f12_sub(f12_sub(f12_sqr(lam), T.x), S.x);
  const Fq12 y3 = f12_sub(f12_mul(lam, f12_sub(T.x, x3)), T.y);
  T.x = x3;
  T.y = y3;
  return l;
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
Fq2 gx(const G2Affine &a) { return Fq2{a.x0, a.x1}; }
Fq2 gy(const G2Affine &a) { return Fq2{a.y0, a.y1}; }
G2Affine mk(const Fq2 &x, const Fq2 &y) {
  G2Affine r;
  r.x0 = x.c0;
  r.x1 = x.c1;
  r.y0 = y.c0;
  r.y1 = y.c1;
  r.inf = false;
  return r;
}
G2Affine g2_inf() {
  G2Affine r;
  r.x0 = r.x1 = r.y0 = r.y1 = Fq::zero();
  r.inf = true;
  return r;
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
    lam = f2_mul(f2_add(f2_add(x2, x2), x2), f2_inv(f2_add(ay, ay)));
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

// k * a for a canonical scalar k (little-endian 64-bit limbs)
G2Affine g2_mul(const G2Affine &a, const uint64_t k[4]) {
  G2Affine r = g2_inf();
  for (int i = 255; i >= 0; i--) {
    r = g2_add(r, r);
    if ((k[i / 64] >> (i % 64)) & 1) r = g2_add(r, a);
  }
  return r;
}

bool g2_on_curve(const G2Affine &a) {
  if (a.inf) return true;
  const Fq2 b = f2_mul(f2(from_u64<FqCfg>(3), Fq::zero()), f2_inv(f2(from_u64<FqCfg>(9), Fq::one())));
  const Fq2 x = gx(a), y = gy(a);
  return f2_eq(f2_sqr(y), f2_add(f2_mul(f2_sqr(x), x), b));
}

// Miller loop value f (before the final exponentiation); 1 for an identity input
static Fq12 miller(const G1Affine &P, const G2Affine &Q) {
  if (P.is_inf() || Q.inf) return f12_one();
  // psi(Q) = (x w^2, y w^3): w^2 = v (Fq6 slot c1 of c0), w^3 = v w (Fq6 slot c1 of c1)
  P12 q;
  q.x = Fq12{Fq6{f2_zero(), gx(Q), f2_zero()}, f6_zero()};
  q.y = Fq12{f6_zero(), Fq6{f2_zero(), gy(Q), f2_zero()}};
  q.inf = false;
  const Fq12 xP = embed_fq(P.x), yP = embed_fq(P.y);
  Fq12 f = f12_one();
  P12 T = q;
  // 6x + 2 = 2^64 + ATE_LOOP: bits below the leading one, high to low
  for (int i = 63; i >= 0; i--) {
    f = f12_mul(f12_sqr(f), line_step(T, T, xP, yP, true));
    if ((ATE_LOOP >> i) & 1) f = f12_mul(f, line_step(T, q, xP, yP, false));
  }
  P12 q1{f12_frob(q.x), f12_frob(q.y), false};  // pi(Q)
  P12 q2{f12_frob(q1.x), f12_neg(f12_frob(q1.y)), false};  // -pi^2(Q)
  f = f12_mul(f, line_step(T, q1, xP, yP, false));
  f = f12_mul(f, line_step(T, q2, xP, yP, false));
  return f;
}

// e(P1, Q1) == e(P2, Q2)
bool pairing_eq(const G1Affine &P1, const G2Affine &Q1, const G1Affine &P2, const G2Affine &Q2) {
  const Fq12 a = final_exp(miller(P1, Q1)), b = final_exp(miller(P2, Q2));
  return f12_eq(a, b);
}

// e(P, Q) as 12 Fq (Montgomery), coefficient order c0.c0.c0, c0.c0.c1, c0.c1.c0, ..., c1.c2.c1
void pairing_value(const G1Affine &P, const G2Affine &Q, Fq out[12]) {
  const Fq12 e = final_exp(miller(P, Q));
  const Fq6 *s[2] = {&e.c0, &e.c1};
  int k = 0;
  for (int i = 0; i < 2; i++) {
    const Fq2 *t[3] = {&s[i]->c0, &s[i]->c1, &s[i]->c2};
    for (int j = 0; j < 3; j++) {
      out[k++] = t[j]->c0;
      out[k++] = t[j]->c1;
    }
  }
}

}  // namespace tns
