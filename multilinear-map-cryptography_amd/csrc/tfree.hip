// tfree.hip -- the Lagrange basis of the nodes {0..N-1} from g1_powers alone (no tau).
//
// The Lagrange route (lagrange.hip) commits to vector_to_polynomial(v) (src/polynomials.rs:301-352)
// as sum_j v_j Lambda_j with Lambda_j = [L_j(tau)]G, and derives the basis from the setup's tau
// (CommitmentParams.tau, src/utils.rs:60-61, :94-100) -- which the reference marks test-only
// (src/utils.rs:61, :107).  Without tau the basis is still a linear image of the SRS:
//
//   Lambda_j = w_j Q_j,   Q_j = [ell(tau) / (tau - j)]G = sum_i q_{j,i} g1_powers[i],
//   ell(x) = prod_{k < N} (x - k),  w_j = (-1)^(N-1-j) / (j! (N-1-j)!)
//
// and all Q_j come out of a TRANSPOSED REMAINDER TREE over the subproduct tree of the nodes
// (the transposition principle applied to multipoint evaluation).  A tree node S = [s, s + m)
// carries the group vector h^S_i = [tau^i ell(tau) / ell_S(tau)]G, i < m, with ell_S the product
// of (x - k) over S.  The root's vector is g1_powers[0..N) itself; a child C with sibling D gets
//
//   h^C_i = sum_{t <= |D|} (ell_D)_t h^S_{i+t},   i < |C|
//
// (ell / ell_C = (ell / ell_S) ell_D), and a leaf {j} holds h_0 = Q_j.  Each level is a batch of
// correlations of group vectors with scalar polynomials: small nodes directly, larger ones by a
// group NTT of the parent vector (DIF: natural in, bit-reversed out), a pointwise scalar
// multiplication by the NTT of each sibling polynomial, and two inverse group NTTs (DIT).  Group
// NTT butterflies multiply points by twiddles -- one variable-base scalar multiplication per
// butterfly, split by the GLV endomorphism into two 127-bit halves walked jointly (xyzz_mul_glv),
// in the lazy domain -- so the build costs ~ 1.5 N log^2 N scalar multiplications: a one-time setup
// per (SRS, N), like the tau-derived basis (tests/test_gpu_tfree.py pins it to that basis; measured
// cost: DESIGN.md 2.8).  The scalar side (the subproduct tree's
// polynomials, stored monic with the leading 1 implicit) is negligible beside it.
#include <hip/hip_runtime.h>

#include <atomic>
#include <thread>
#include <vector>

#include "common.hpp"
#include "ntt.hpp"

namespace tns {

namespace {

constexpr size_t TF_DIRECT_H = 4;  // children of <= 4 nodes: direct correlation (h scalar mults / output)
// the kernels that multiply points by scalars: 3 waves per SIMD (168 VGPRs; the default bound let
// the compiler take 258 registers, one wave per SIMD)
#define TF_WAVES 3
// the group NTT's butterflies (GLV joint multiplication: P, phi(P), their sum and the accumulator)
#ifndef TF_NTT_WAVES
#define TF_NTT_WAVES 2
#endif

__device__ __forceinline__ G1Xyzz xyzz_negate(const G1Xyzz &p) {
  G1Xyzz r = p;
  r.y = neg(p.y);
  return r;
}

// dbl-2008-s-1 in the lazy domain (coordinates in [0, 2M), as xyzz_add_lazy): no final
// subtractions in the products, Y3 as one reduction of M (S - X3) + Y (2M - W)
__device__ __forceinline__ G1Xyzz xyzz_dbl_lazy(const G1Xyzz &p) {
  if (fq_zero_lazy(p.zz) || fq_zero_lazy(p.y)) return G1Xyzz::inf();
  const Fq U = add2_dev(p.y, p.y);
  const Fq V = sqr_lazy_dev(U);
  const Fq W = mul_lazy_dev(U, V);
  const Fq S = mul_lazy_dev(p.x, V);
  const Fq X2 = sqr_lazy_dev(p.x);
  const Fq M = add2_dev(add2_dev(X2, X2), X2);
  G1Xyzz r;
  r.x = sub2_dev(sqr_lazy_dev(M), add2_dev(S, S));
  r.y = mul2_lazy_dev(M, sub2_dev(S, r.x), p.y, const_minus_dev<FqCfg, true>(W));
  r.zz = mul_lazy_dev(V, p.zz);
  r.zzz = mul_lazy_dev(W, p.zzz);
  return r;
}

// k P for a canonical scalar k: left to right from k's top bit.  Where the lanes of a wave share
// k (the group NTT maps equal twiddles to one wave), the branches are uniform.
__device__ G1Xyzz xyzz_mul_canon(const G1Xyzz &P, const Fr &k) {
  G1Xyzz acc = G1Xyzz::inf();
  bool started = false;
#pragma unroll 1
  for (int l = 7; l >= 0; l--) {
    uint32_t w = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) w = q == l ? k.v[q] : w;  // (a dynamic index would use scratch)
    if (!started && w == 0) continue;
#pragma unroll 1
    for (int b = 31; b >= 0; b--) {
      if (started) acc = xyzz_dbl_lazy(acc);
      if ((w >> b) & 1u) {
        acc = started ? xyzz_add_lazy(acc, P) : P;
        started = true;
      }
    }
  }
  return xyzz_canon(acc);
}

// ---- GLV: phi(x, y) = (beta x, y) equals lambda (x, y) on G1 (beta a primitive cube root of unity
// in Fq, lambda the matching one in Fr: phi(G) = lambda G, checked against the C oracle when the
// constants were derived), so k P = k1 P + k2 phi(P) with k = k1 + k2 lambda (mod r) and
// |k1|, |k2| < 2^127: half the doublings of a 254-bit double-and-add.  The group NTT's twiddles are
// split once per basis build on the host (Babai rounding in the reduced lattice basis
// (a1, b1), (a2, b2) of {(a, b): a + b lambda = 0 mod r}; g1 = floor(b2 2^256 / r),
// g2 = floor(-b1 2^256 / r)).
struct GlvScalar {
  uint32_t k1[4], k2[4];  // magnitudes
  uint32_t neg;           // bit 0: k1 < 0, bit 1: k2 < 0
};
// beta in Montgomery form (canonical 0x30644e72e131a0295e6dd9e7e0acccb0c28f069fbb966e3de4bd44e5607cfd48)
__constant__ uint32_t kGlvBeta[8] = {0x13e80b9cu, 0x3350c88eu, 0xdb5e56b9u, 0x7dce557cu,
                                     0xb615564au, 0x6001b4b8u, 0x020217e0u, 0x2682e617u};

// k1 P + k2 phi(P), joint left-to-right double-and-add (Straus-Shamir: P, phi(P) and their sum)
// from bit 126; uniform per wave where the lanes share the scalar (the twiddles)
__device__ G1Xyzz xyzz_mul_glv(const G1Xyzz &P, const GlvScalar &s) {
  const G1Xyzz P1 = (s.neg & 1u) ? xyzz_negate(P) : P;
  Fq beta;
#pragma unroll
  for (int q = 0; q < 8; q++) beta.v[q] = kGlvBeta[q];
  G1Xyzz P2 = P;
  P2.x = mul(P.x, beta);
  if (s.neg & 2u) P2.y = neg(P.y);
  const G1Xyzz P12 = xyzz_add(P1, P2);  // Straus-Shamir: one addition where both bits are set
  G1Xyzz acc = G1Xyzz::inf();
  bool started = false;
#pragma unroll 1
  for (int l = 3; l >= 0; l--) {
    uint32_t w1 = 0, w2 = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {  // (a dynamic index would use scratch)
      w1 = q == l ? s.k1[q] : w1;
      w2 = q == l ? s.k2[q] : w2;
    }
    if (!started && (w1 | w2) == 0) continue;
#pragma unroll 1
    for (int b = 31; b >= 0; b--) {
      if (started) acc = xyzz_dbl_lazy(acc);
      const uint32_t d = ((w1 >> b) & 1u) | (((w2 >> b) & 1u) << 1);
      if (d) {
        const G1Xyzz &T = d == 3 ? P12 : d == 1 ? P1 : P2;
        acc = started ? xyzz_add_lazy(acc, T) : T;
        started = true;
      }
    }
  }
  return xyzz_canon(acc);  // the butterflies' canonical additions read it
}

// host: the lattice constants (64-bit limbs, little endian)
static const uint64_t kGlvA1[2] = {0x8211bbeb7d4f1128ull, 0x6f4d8248eeb859fcull};
static const uint64_t kGlvA2[1] = {0x89d3256894d213e3ull};
static const uint64_t kGlvB1Abs[1] = {0x89d3256894d213e3ull};
static const uint64_t kGlvB2[2] = {0x0be4e1541221250bull, 0x6f4d8248eeb859fdull};
static const uint64_t kGlvG1[3] = {0x5398fd0300ff6565ull, 0x4ccef014a773d2d2ull, 0x2ull};
static const uint64_t kGlvG2[2] = {0xd91d232ec7e0b3d7ull, 0x2ull};

static void limbs_mul(const uint64_t *a, int na, const uint64_t *b, int nb, uint64_t *r) {  // r: na + nb limbs
  for (int i = 0; i < na + nb; i++) r[i] = 0;
  for (int i = 0; i < na; i++) {
    unsigned __int128 c = 0;
    for (int j = 0; j < nb; j++) {
      c += (unsigned __int128)a[i] * b[j] + r[i + j];
      r[i + j] = (uint64_t)c;
      c >>= 64;
    }
    r[i + nb] = (uint64_t)c;
  }
}

// |a - b| into r (n limbs); returns a < b
static bool limbs_absdiff(const uint64_t *a, const uint64_t *b, uint64_t *r, int n) {
  int c = 0;
  for (int i = n - 1; i >= 0 && !c; i--) c = a[i] < b[i] ? -1 : a[i] > b[i] ? 1 : 0;
  const uint64_t *x = c < 0 ? b : a, *y = c < 0 ? a : b;
  unsigned __int128 br = 0;
  for (int i = 0; i < n; i++) {
    const unsigned __int128 d = (unsigned __int128)x[i] - y[i] - br;
    r[i] = (uint64_t)d;
    br = (d >> 64) & 1;
  }
  return c < 0;
}

// canonical k < r -> (k1, k2); throws if a part exceeds 128 bits (it cannot: |k1|, |k2| < 2^127)
static GlvScalar glv_split(const uint64_t k[4]) {
  uint64_t p1[7], p2[6];
  limbs_mul(k, 4, kGlvG1, 3, p1);
  limbs_mul(k, 4, kGlvG2, 2, p2);
  const uint64_t c1[3] = {p1[4], p1[5], p1[6]}, c2[2] = {p2[4], p2[5]};
  uint64_t t1[5], t2[3], t[5], kk[5] = {k[0], k[1], k[2], k[3], 0}, k1[5];
  limbs_mul(c1, 3, kGlvA1, 2, t1);
  limbs_mul(c2, 2, kGlvA2, 1, t2);
  unsigned __int128 cy = 0;
  for (int i = 0; i < 5; i++) {
    cy += (unsigned __int128)t1[i] + (i < 3 ? t2[i] : 0);
    t[i] = (uint64_t)cy;
    cy >>= 64;
  }
  const bool n1 = limbs_absdiff(kk, t, k1, 5);
  uint64_t u1[4], u2[4], k2[4];
  limbs_mul(c1, 3, kGlvB1Abs, 1, u1);
  limbs_mul(c2, 2, kGlvB2, 2, u2);
  const bool n2 = limbs_absdiff(u1, u2, k2, 4);
  if (k1[2] | k1[3] | k1[4] | k2[2] | k2[3]) throw Error(TNS_ERR_INVALID_PARAMETERS, "GLV split out of range");
  GlvScalar g;
  for (int i = 0; i < 2; i++) {
    g.k1[2 * i] = (uint32_t)k1[i];
    g.k1[2 * i + 1] = (uint32_t)(k1[i] >> 32);
    g.k2[2 * i] = (uint32_t)k2[i];
    g.k2[2 * i + 1] = (uint32_t)(k2[i] >> 32);
  }
  g.neg = (n1 ? 1u : 0u) | (n2 ? 2u : 0u);
  return g;
}

__global__ void __launch_bounds__(256) k_tf_canon_twiddles(const Fr *__restrict__ TW, size_t n, Fr *__restrict__ out) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = from_mont(TW[i]);
}

// the twiddle table TW[0..N) split for the group NTT (download, split on host threads, upload)
static void glv_twiddles(Ctx *c, const Fr *TW, size_t N, DevBuf &out) {
  DevBuf canon;
  Fr *d_canon = (Fr *)canon.ensure(sizeof(Fr) * N);
  k_tf_canon_twiddles<<<grid_for(N, 256, 4096), 256, 0, c->stream>>>(TW, N, d_canon);
  TNS_LAUNCH_CHECK();
  std::vector<Fr> h(N);
  TNS_HIP(hipMemcpyAsync(h.data(), d_canon, sizeof(Fr) * N, hipMemcpyDeviceToHost, c->stream));
  TNS_HIP(hipStreamSynchronize(c->stream));
  std::vector<GlvScalar> g(N);
  const size_t nt = std::max<size_t>(1, std::min<size_t>(16, N / 4096));
  std::vector<std::thread> ths;
  std::atomic<bool> bad(false);
  auto work = [&](size_t t) {
    for (size_t i = t; i < N; i += nt) {
      uint64_t k[4];
      for (int q = 0; q < 4; q++) k[q] = (uint64_t)h[i].v[2 * q] | ((uint64_t)h[i].v[2 * q + 1] << 32);
      try {
        g[i] = glv_split(k);
      } catch (...) {
        bad = true;
      }
    }
  };
  try {
    for (size_t t = 1; t < nt; t++) ths.emplace_back(work, t);
  } catch (...) {  // threads that could not start: their share runs here
    for (size_t t = ths.size() + 1; t < nt; t++) work(t);
  }
  work(0);
  for (auto &th : ths) th.join();
  if (bad) throw Error(TNS_ERR_INVALID_PARAMETERS, "GLV split out of range");
  GlvScalar *d = (GlvScalar *)out.ensure(sizeof(GlvScalar) * N);
  TNS_HIP(hipMemcpyAsync(d, g.data(), sizeof(GlvScalar) * N, hipMemcpyHostToDevice, c->stream));
  TNS_HIP(hipStreamSynchronize(c->stream));
}

// ---- scalar side: the subproduct tree ell_S, monic, leading coefficient implicit.  Level e holds
// the N / 2^e nodes of size h = 2^e, node k's h coefficients at [k h, (k + 1) h).
__global__ void __launch_bounds__(256) k_tf_leaves(size_t N, Fr *__restrict__ L0) {
  for (size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < N; k += (size_t)gridDim.x * blockDim.x)
    L0[k] = neg(from_u64<FrCfg>((uint64_t)k));  // x - k
}

// parent p = (x^h + a)(x^h + b) = x^2h + x^h (a + b) + a b, directly (small h)
__global__ void __launch_bounds__(256) k_tf_poly_direct(const Fr *__restrict__ Lin, size_t N, size_t h,
                                                        Fr *__restrict__ Lout) {
  for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < N; idx += (size_t)gridDim.x * blockDim.x) {
    const size_t p = idx / (2 * h), i = idx - p * 2 * h;
    const Fr *a = Lin + 2 * p * h, *b = a + h;
    Fr s = Fr::zero();
    const size_t u0 = i >= h ? i - h + 1 : 0, u1 = i < h ? i : h - 1;
    for (size_t u = u0; u <= u1; u++) s = add(s, mul(a[u], b[i - u]));
    if (i >= h) s = add(s, add(a[i - h], b[i - h]));
    Lout[idx] = s;
  }
}

// batched radix-2 NTT stages over arrays of N entries holding N / M transforms of size M each
// (blocks of 2 hs never cross a transform).  TW: ntt_twiddles layout, TW[hs + j] = w_{2hs}^j.
// Thread t -> (j = t / nB, block B = t % nB): consecutive lanes share the twiddle j.
__global__ void __launch_bounds__(256) k_tf_fdif(Fr *__restrict__ X, size_t N, size_t hs, const Fr *__restrict__ TW) {
  const size_t nB = N / (2 * hs), half = N / 2;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < half; t += (size_t)gridDim.x * blockDim.x) {
    const size_t j = t / nB, a = (t - j * nB) * 2 * hs + j, b = a + hs;
    const Fr x = X[a], y = X[b];
    X[a] = add(x, y);
    X[b] = mul(sub(x, y), TW[hs + j]);
  }
}
// inverse (bit-reversed in, natural out, unscaled): w^-j = -TW[2 hs - j]
__global__ void __launch_bounds__(256) k_tf_fdit(Fr *__restrict__ X, size_t N, size_t hs, const Fr *__restrict__ TW) {
  const size_t nB = N / (2 * hs), half = N / 2;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < half; t += (size_t)gridDim.x * blockDim.x) {
    const size_t j = t / nB, a = (t - j * nB) * 2 * hs + j, b = a + hs;
    const Fr x = X[a];
    const Fr y = j ? neg(mul(X[b], TW[2 * hs - j])) : X[b];
    X[a] = add(x, y);
    X[b] = sub(x, y);
  }
}
__global__ void __launch_bounds__(256, TF_NTT_WAVES) k_tf_gdif(G1Xyzz *__restrict__ X, size_t N, size_t hs,
                                                 const GlvScalar *__restrict__ TG) {
  const size_t nB = N / (2 * hs), half = N / 2;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < half; t += (size_t)gridDim.x * blockDim.x) {
    const size_t j = t / nB, a = (t - j * nB) * 2 * hs + j, b = a + hs;
    const G1Xyzz x = X[a], y = X[b];
    X[a] = xyzz_add(x, y);
    const G1Xyzz d = xyzz_add(x, xyzz_negate(y));
    X[b] = j ? xyzz_mul_glv(d, TG[hs + j]) : d;
  }
}
__global__ void __launch_bounds__(256, TF_NTT_WAVES) k_tf_gdit(G1Xyzz *__restrict__ X, size_t N, size_t hs,
                                                 const GlvScalar *__restrict__ TG) {
  const size_t nB = N / (2 * hs), half = N / 2;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < half; t += (size_t)gridDim.x * blockDim.x) {
    const size_t j = t / nB, a = (t - j * nB) * 2 * hs + j, b = a + hs;
    const G1Xyzz x = X[a];
    const G1Xyzz y = j ? xyzz_negate(xyzz_mul_glv(X[b], TG[2 * hs - j])) : X[b];
    X[a] = xyzz_add(x, y);
    X[b] = xyzz_add(x, xyzz_negate(y));
  }
}

static void fr_ntt(hipStream_t st, Fr *X, size_t N, size_t M, const Fr *TW, bool inverse) {
  const unsigned g = grid_for(N / 2, 256, 1u << 20);
  if (!inverse) {
    for (size_t hs = M / 2; hs >= 1; hs /= 2) k_tf_fdif<<<g, 256, 0, st>>>(X, N, hs, TW);
  } else {
    for (size_t hs = 1; hs < M; hs *= 2) k_tf_fdit<<<g, 256, 0, st>>>(X, N, hs, TW);
  }
  TNS_LAUNCH_CHECK();
}

// a -> A (padded to 2h), b -> B, per parent
__global__ void __launch_bounds__(256) k_tf_pad2(const Fr *__restrict__ Lin, size_t N, size_t h, Fr *__restrict__ A,
                                                 Fr *__restrict__ B) {
  for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < N; idx += (size_t)gridDim.x * blockDim.x) {
    const size_t p = idx / (2 * h), i = idx - p * 2 * h;
    A[idx] = i < h ? Lin[2 * p * h + i] : Fr::zero();
    B[idx] = i < h ? Lin[2 * p * h + h + i] : Fr::zero();
  }
}
__global__ void __launch_bounds__(256) k_tf_pmul(Fr *__restrict__ A, const Fr *__restrict__ B, size_t N, Fr s) {
  for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < N; idx += (size_t)gridDim.x * blockDim.x)
    A[idx] = mul(mul(A[idx], B[idx]), s);
}
// Lout = a b (in A, 2h coefficients, the top one zero) + x^h (a + b)
__global__ void __launch_bounds__(256) k_tf_poly_finish(const Fr *__restrict__ Lin, const Fr *__restrict__ AB, size_t N,
                                                        size_t h, Fr *__restrict__ Lout) {
  for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < N; idx += (size_t)gridDim.x * blockDim.x) {
    const size_t p = idx / (2 * h), i = idx - p * 2 * h;
    Fr s = AB[idx];
    if (i >= h) s = add(s, add(Lin[2 * p * h + i - h], Lin[2 * p * h + h + i - h]));
    Lout[idx] = s;
  }
}

// ---- group side, one tree level: node size M = 2h, children 2k (left) and 2k + 1 (right) of node k
// direct: out[kM + i] = h^{left}_i (coefficients of the RIGHT child), out[kM + h + i] = h^{right}_i
__global__ void __launch_bounds__(256, TF_WAVES) k_tf_level_direct(const G1Xyzz *__restrict__ H, const Fr *__restrict__ Lc,
                                                         size_t N, size_t h, G1Xyzz *__restrict__ out) {
  const size_t M = 2 * h;
  for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < N; idx += (size_t)gridDim.x * blockDim.x) {
    const size_t k = idx / M, r = idx - k * M;
    const bool left = r < h;
    const size_t i = left ? r : r - h;
    const Fr *c = Lc + (2 * k + (left ? 1 : 0)) * h;  // the sibling's ell
    const G1Xyzz *in = H + k * M + i;
    G1Xyzz acc = in[h];  // leading coefficient 1
    for (size_t t = 0; t < h; t++) acc = xyzz_add(acc, xyzz_mul_canon(in[t], from_mont(c[t])));
    out[idx] = acc;
  }
}

// the two children's correlation kernels, reversed into cyclic length M (cp_k = c_{h-k}, k <= h)
__global__ void __launch_bounds__(256) k_tf_rev_pad(const Fr *__restrict__ Lc, size_t N, size_t h,
                                                    Fr *__restrict__ SL, Fr *__restrict__ SR) {
  const size_t M = 2 * h;
  for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < N; idx += (size_t)gridDim.x * blockDim.x) {
    const size_t k = idx / M, r = idx - k * M;
    Fr l = Fr::zero(), rr = Fr::zero();
    if (r == 0) {
      l = rr = Fr::one();
    } else if (r <= h) {
      l = Lc[2 * k * h + (h - r)];
      rr = Lc[(2 * k + 1) * h + (h - r)];
    }
    SL[idx] = l;
    SR[idx] = rr;
  }
}
// spectra: scaled by 1/M and made canonical (the scalar multiplications read their bits)
__global__ void __launch_bounds__(256) k_tf_scale_canon(Fr *__restrict__ S, size_t N, Fr s) {
  for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < N; idx += (size_t)gridDim.x * blockDim.x)
    S[idx] = from_mont(mul(S[idx], s));
}
// Y[idx] = H^[idx] * SR[idx] (left child), H^[idx] *= SL[idx] (right child), in bit-reversed order
__global__ void __launch_bounds__(256, TF_NTT_WAVES) k_tf_pointwise(G1Xyzz *__restrict__ Hh, const Fr *__restrict__ SL,
                                                      const Fr *__restrict__ SR, size_t N, G1Xyzz *__restrict__ Y) {
  for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < N; idx += (size_t)gridDim.x * blockDim.x) {
    const G1Xyzz p = Hh[idx];
    Y[idx] = xyzz_mul_canon(p, SR[idx]);
    Hh[idx] = xyzz_mul_canon(p, SL[idx]);
  }
}
// out[kM + i] = left[kM + h + i], out[kM + h + i] = right[kM + h + i]  (conv index i + h)
__global__ void __launch_bounds__(256) k_tf_take(const G1Xyzz *__restrict__ Yl, const G1Xyzz *__restrict__ Yr,
                                                 size_t N, size_t h, G1Xyzz *__restrict__ out) {
  const size_t M = 2 * h;
  for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < N; idx += (size_t)gridDim.x * blockDim.x) {
    const size_t r = idx % M;
    out[idx] = r < h ? Yl[idx + h] : Yr[idx];
  }
}

static void g_ntt(hipStream_t st, G1Xyzz *X, size_t N, size_t M, const GlvScalar *TG, bool inverse) {
  const unsigned g = grid_for(N / 2, 256, 1u << 20);
  if (!inverse) {
    for (size_t hs = M / 2; hs >= 1; hs /= 2) k_tf_gdif<<<g, 256, 0, st>>>(X, N, hs, TG);
  } else {
    for (size_t hs = 1; hs < M; hs *= 2) k_tf_gdit<<<g, 256, 0, st>>>(X, N, hs, TG);
  }
  TNS_LAUNCH_CHECK();
}

__global__ void __launch_bounds__(256) k_tf_from_affine(const G1Affine *__restrict__ g, size_t N,
                                                        G1Xyzz *__restrict__ H) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < N; i += (size_t)gridDim.x * blockDim.x)
    H[i] = xyzz_from_affine(g[i]);
}
// Lambda_j = w_j Q_j
__global__ void __launch_bounds__(256, TF_WAVES) k_tf_weights(G1Xyzz *__restrict__ H, const Fr *__restrict__ w, size_t N) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < N; i += (size_t)gridDim.x * blockDim.x)
    H[i] = xyzz_mul_canon(H[i], from_mont(w[i]));
}

}  // namespace

const LagrangeBasis *lagrange_basis_from_powers_dev(Ctx *c, const Srs &srs, size_t N) {
  if (N == 0 || (N & (N - 1))) throw Error(TNS_ERR_INVALID_PARAMETERS, "Lagrange basis size must be a power of two");
  if (N > ((size_t)1 << 28)) throw Error(TNS_ERR_INVALID_PARAMETERS, "Lagrange basis larger than 2^28");
  if (srs.first != 0 || srs.held < N)
    throw Error(TNS_ERR_INVALID_PARAMETERS, "the basis of N nodes needs g1_powers[0..N) (an unsharded SRS)");
  const auto key = std::make_tuple(N, (size_t)0, N);
  auto it = srs.lagrange.find(key);
  if (it != srs.lagrange.end()) return it->second;
  hipStream_t st = c->stream;
  const unsigned n = ilog2_exact(N);
  const G1Affine *g = srs.points.as<G1Affine>();
  LagrangeBasis *basis = new LagrangeBasis();
  try {
    G1Affine *pts = (G1Affine *)basis->points.ensure(sizeof(G1Affine) * N);
    if (N == 1) {  // L_0 = 1
      TNS_HIP(hipMemcpyAsync(pts, g, sizeof(G1Affine), hipMemcpyDeviceToDevice, st));
    } else {
      const Fr *TW = ntt_twiddles(c, n);
      // scalar side: every level of the subproduct tree (children of size h = 2^e, e < n)
      DevBuf lcb, ab, bb;
      Fr *Lc = (Fr *)lcb.ensure(sizeof(Fr) * N * n);
      const unsigned gN = grid_for(N, 256, 1u << 20);
      k_tf_leaves<<<gN, 256, 0, st>>>(N, Lc);
      TNS_LAUNCH_CHECK();
      Fr *A = (Fr *)ab.ensure(sizeof(Fr) * N), *B = (Fr *)bb.ensure(sizeof(Fr) * N);
      for (unsigned e = 0; e + 1 < n; e++) {
        const size_t h = (size_t)1 << e;
        const Fr *Lin = Lc + (size_t)e * N;
        Fr *Lout = Lc + (size_t)(e + 1) * N;
        if (h <= 32) {
          k_tf_poly_direct<<<gN, 256, 0, st>>>(Lin, N, h, Lout);
          TNS_LAUNCH_CHECK();
        } else {  // a b by a cyclic product of length 2h (deg a b <= 2h - 2: no wrap)
          k_tf_pad2<<<gN, 256, 0, st>>>(Lin, N, h, A, B);
          TNS_LAUNCH_CHECK();
          fr_ntt(st, A, N, 2 * h, TW, false);
          fr_ntt(st, B, N, 2 * h, TW, false);
          k_tf_pmul<<<gN, 256, 0, st>>>(A, B, N, inv(from_u64<FrCfg>((uint64_t)(2 * h))));
          TNS_LAUNCH_CHECK();
          fr_ntt(st, A, N, 2 * h, TW, true);
          k_tf_poly_finish<<<gN, 256, 0, st>>>(Lin, A, N, h, Lout);
          TNS_LAUNCH_CHECK();
        }
      }
      // group side, root to leaves: H holds every node's vector of the current level
      DevBuf tgb;
      glv_twiddles(c, TW, N, tgb);
      const GlvScalar *TG = tgb.as<GlvScalar>();
      DevBuf hb, hh, yb;
      G1Xyzz *H = (G1Xyzz *)hb.ensure(sizeof(G1Xyzz) * N), *Hh = (G1Xyzz *)hh.ensure(sizeof(G1Xyzz) * N);
      k_tf_from_affine<<<gN, 256, 0, st>>>(g, N, H);
      TNS_LAUNCH_CHECK();
      const unsigned gS = grid_for(N, 256, 4096);  // scalar-multiplication kernels: whole waves of work
      G1Xyzz *Y = nullptr;
      for (int e = (int)n - 1; e >= 0; e--) {
        const size_t h = (size_t)1 << e, M = 2 * h;
        const Fr *Le = Lc + (size_t)e * N;  // the children's ell
        if (h <= TF_DIRECT_H) {
          k_tf_level_direct<<<gS, 256, 0, st>>>(H, Le, N, h, Hh);
          TNS_LAUNCH_CHECK();
          std::swap(H, Hh);
          continue;
        }
        if (!Y) Y = (G1Xyzz *)yb.ensure(sizeof(G1Xyzz) * N);
        k_tf_rev_pad<<<gN, 256, 0, st>>>(Le, N, h, A, B);  // A = SL (left child's ell), B = SR
        TNS_LAUNCH_CHECK();
        fr_ntt(st, A, N, M, TW, false);
        fr_ntt(st, B, N, M, TW, false);
        const Fr iM = inv(from_u64<FrCfg>((uint64_t)M));
        k_tf_scale_canon<<<gN, 256, 0, st>>>(A, N, iM);
        k_tf_scale_canon<<<gN, 256, 0, st>>>(B, N, iM);
        TNS_LAUNCH_CHECK();
        TNS_HIP(hipMemcpyAsync(Hh, H, sizeof(G1Xyzz) * N, hipMemcpyDeviceToDevice, st));
        g_ntt(st, Hh, N, M, TG, false);
        k_tf_pointwise<<<gS, 256, 0, st>>>(Hh, A, B, N, Y);  // Y: left child (SR), Hh: right child (SL)
        TNS_LAUNCH_CHECK();
        g_ntt(st, Y, N, M, TG, true);
        g_ntt(st, Hh, N, M, TG, true);
        k_tf_take<<<gN, 256, 0, st>>>(Y, Hh, N, h, H);
        TNS_LAUNCH_CHECK();
      }
      // H[j] = Q_j;  Lambda_j = w_j Q_j, then affine
      k_tf_weights<<<gS, 256, 0, st>>>(H, bary_weights_dev(c, N, 0, N), N);
      TNS_LAUNCH_CHECK();
      DevBuf pre;
      xyzz_to_affine_batch_dev(c, H, N, pts, (Fq *)pre.ensure(sizeof(Fq) * N));
      TNS_HIP(hipStreamSynchronize(st));
    }
    if (N >= ((size_t)1 << 12)) basis->fb = fixed_base_try_build(c, pts, N);
    TNS_HIP(hipStreamSynchronize(st));
  } catch (...) {
    delete basis;
    throw;
  }
  srs.lagrange[key] = basis;
  return basis;
}

}  // namespace tns
