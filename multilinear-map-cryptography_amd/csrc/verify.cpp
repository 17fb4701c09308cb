// verify.cpp -- the verifiers of the reference, on the host:
//   KZGCommitment::verify / batch_verify   src/commitments.rs:201-301
//   SumCheck::verify                       src/sumcheck.rs:113-150
//   Twist::verify, Shout::verify           src/twist.rs:255-304, src/shout.rs:225-274
//   CommitmentVerificationKey              src/utils.rs:64-75, :104-112 (g2_tau = tau * G2)
// Restated step by step, including batch_verify's pairing equation exactly as written
// (e(sum g_i (C_i - v_i G), G2) == e(sum g_i pi_i, sum g_i (tau - z_i) G2) with the g_i drawn
// from ChaCha20Rng([42;32])), so that every boolean matches the reference's.
#include <cstring>
#include <vector>

#include "common.hpp"
#include "hostfield.hpp"

namespace tns {

static void canon64(const Fr &x, uint64_t out[4]) {
  const Fr c = from_mont(x);
  for (int i = 0; i < 4; i++) out[i] = (uint64_t)c.v[2 * i] | ((uint64_t)c.v[2 * i + 1] << 32);
}

// k * P on the host: double-and-add over XYZZ in the 4 x u64 host field (hostfield.hpp),
// k a Montgomery-form Fr.  dbl-2008-s-1 / madd-2008-s (a = 0).
namespace {
struct HX {
  HFq x, y, zz, zzz;
};
HX hx_dbl(const HX &p) {
  if (p.zz.is_zero()) return p;
  const HFq U = p.y + p.y, V = U * U, W = U * V, S = p.x * V;
  const HFq X2 = p.x * p.x, M = X2 + X2 + X2;
  const HFq X3 = M * M - (S + S);
  return HX{X3, M * (S - X3) - W * p.y, V * p.zz, W * p.zzz};
}
HX hx_madd(const HX &p, const HFq &x2, const HFq &y2) {
  if (p.zz.is_zero()) return HX{x2, y2, HFq::one(), HFq::one()};
  const HFq P = x2 * p.zz - p.x, R = y2 * p.zzz - p.y;
  if (P.is_zero()) {
    if (R.is_zero()) return hx_dbl(HX{x2, y2, HFq::one(), HFq::one()});
    return HX{HFq::one(), HFq::one(), HFq::zero(), HFq::zero()};
  }
  const HFq PP = P * P, PPP = P * PP, Q = p.x * PP;
  const HFq X3 = R * R - PPP - (Q + Q);
  return HX{X3, R * (Q - X3) - p.y * PPP, p.zz * PP, p.zzz * PPP};
}
}  // namespace

G1Xyzz g1_mul_host(const G1Affine &P, const Fr &k) {
  if (P.is_inf()) return G1Xyzz::inf();
  uint64_t e[4];
  canon64(k, e);
  const HFq px = HFq::of(P.x), py = HFq::of(P.y);
  HX r{HFq::one(), HFq::one(), HFq::zero(), HFq::zero()};
  for (int i = 255; i >= 0; i--) {
    r = hx_dbl(r);
    if ((e[i / 64] >> (i % 64)) & 1) r = hx_madd(r, px, py);
  }
  if (r.zz.is_zero()) return G1Xyzz::inf();
  G1Xyzz out;
  out.x = r.x.fp();
  out.y = r.y.fp();
  out.zz = r.zz.fp();
  out.zzz = r.zzz.fp();
  return out;
}

G1Affine g1_generator_host() {
  G1Affine g;
  g.x = from_u64<FqCfg>(1);
  g.y = from_u64<FqCfg>(2);
  return g;
}

void verifier_key(const Fr &tau, G1Affine *g1, G2Affine *g2, G2Affine *g2_tau) {
  *g1 = g1_generator_host();
  *g2 = g2_generator();
  uint64_t t[4];
  canon64(tau, t);
  *g2_tau = g2_mul(*g2, t);
}

// e(C - v G1, G2) == e(pi, tau G2 - z G2)   (src/commitments.rs:201-228)
bool kzg_verify_host(const G1Affine &g1, const G2Affine &g2, const G2Affine &g2_tau, const G1Affine &C,
                     const Fr &z, const Fr &v, const G1Affine &pi) {
  const G1Xyzz left = xyzz_add(xyzz_from_affine(C), g1_mul_host(g1_neg(g1), v));
  uint64_t zc[4];
  canon64(z, zc);
  const G2Affine right = g2_add(g2_tau, g2_neg(g2_mul(g2, zc)));
  return pairing_eq(xyzz_to_affine(left), g2, pi, right);
}

// src/commitments.rs:230-301 (empty input -> true; lengths are checked by the caller)
bool kzg_batch_verify_host(const G1Affine &g1, const G2Affine &g2, const G2Affine &g2_tau, size_t n,
                           const G1Affine *C, const Fr *z, const Fr *v, const G1Affine *pi) {
  if (n == 0) return true;
  uint8_t seed42[32];
  std::memset(seed42, 42, 32);
  std::vector<Fr> gam(n);
  host_fr_rand_stream(seed42, n, gam.data());
  G1Xyzz bc = G1Xyzz::inf(), bp = G1Xyzz::inf();
  Fr bv = Fr::zero();
  G2Affine bg2;
  bg2.x0 = bg2.x1 = bg2.y0 = bg2.y1 = Fq::zero();
  bg2.inf = true;
  for (size_t i = 0; i < n; i++) {
    bc = xyzz_add(bc, g1_mul_host(C[i], gam[i]));
    bv = add(bv, mul(v[i], gam[i]));
    bp = xyzz_add(bp, g1_mul_host(pi[i], gam[i]));
    uint64_t zc[4], gc[4];
    canon64(z[i], zc);
    canon64(gam[i], gc);
    const G2Affine t = g2_add(g2_tau, g2_neg(g2_mul(g2, zc)));
    bg2 = g2_add(bg2, g2_mul(t, gc));
  }
  const G1Xyzz left = xyzz_add(bc, g1_mul_host(g1_neg(g1), bv));
  return pairing_eq(xyzz_to_affine(left), g2, xyzz_to_affine(bp), bg2);
}

// SumCheck::verify with claimed sum 0 (src/sumcheck.rs:113-150); round polynomials are
// 4 coefficients (evaluate_round_polynomial = Horner, :209-212)
bool sumcheck_verify_host(HostTranscript &tr, const Fr *rounds, unsigned nv, const Fr &final_eval) {
  Fr cur = Fr::zero();
  char lab[64];
  for (unsigned r = 0; r < nv; r++) {
    const Fr *c = rounds + 4 * (size_t)r;
    const Fr g0 = horner_host(c, 4, Fr::zero()), g1 = horner_host(c, 4, Fr::one());
    if (add(g0, g1) != cur) return false;
    snprintf(lab, sizeof lab, "sumcheck_round_%u", r);
    tr.append_label(lab);
    for (int x = 0; x < 4; x++) tr.append_fr(c[x]);
    snprintf(lab, sizeof lab, "sumcheck_challenge_%u", r);
    const Fr ch = tr.challenge(lab);
    cur = horner_host(c, 4, ch);
  }
  return cur == final_eval;
}

// Twist::verify / Shout::verify: labels of the two commitments differ
bool protocol_verify_host(const G1Affine &g1, const G2Affine &g2, const G2Affine &g2_tau, const char *label0,
                          const char *label1, const G1Affine C[2], const Fr *rounds, unsigned nv,
                          const Fr &final_eval, unsigned n_openings, const G1Affine pi[2], const Fr vals[2]) {
  HostTranscript tr;
  tr.append_label(label0);
  tr.append_fr(commitment_hash(C[0]));
  tr.append_label(label1);
  tr.append_fr(commitment_hash(C[1]));
  if (!sumcheck_verify_host(tr, rounds, nv, final_eval)) return false;
  if (nv == 0 || n_openings < 2) return true;  // challenge_field_elements(.., 0) is empty
  Fr z = tr.challenge("opening_challenges_0");
  char lab[64];
  for (unsigned i = 1; i < nv; i++) {
    snprintf(lab, sizeof lab, "opening_challenges_%u", i);
    (void)tr.challenge(lab);
  }
  for (int k = 0; k < 2; k++)
    if (!kzg_verify_host(g1, g2, g2_tau, C[k], z, vals[k], pi[k])) return false;
  return true;
}

}  // namespace tns
