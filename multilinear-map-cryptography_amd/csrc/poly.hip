// poly.hip -- univariate helpers on the device: synthetic division (KZG open),
// SRS generation (setup_params), and element conversions.
//
// KZG open (src/commitments.rs:182-199, :305-375): the reference evaluates v = P(z)
// by Horner and then long-divides (P - v) by (x - z).  Both are the same linear
// recurrence
//     s_n = 0,   s_j = c_j + z * s_{j+1}      (j = n-1 .. 0)
// with v = s_0 and quotient q_i = s_{i+1}.  We evaluate it as a parallel suffix
// scan: chunks of K coefficients run the recurrence locally, the chunk carries
// obey the same recurrence with multiplier z^K (solved recursively), and a final
// pass replays each chunk with its carry.  HBM traffic: read c twice, write s once.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "common.hpp"

namespace tns {

constexpr int SCAN_K = 64;

// L_j = sum_{t in chunk j} c_t z^(t - jK)
__global__ void __launch_bounds__(256) k_scan_chunk_local(const Fr *__restrict__ c, size_t n, Fr z,
                                                          Fr *__restrict__ L, size_t C) {
  size_t j = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (j >= C) return;
  size_t a = j * SCAN_K, b = a + SCAN_K;
  if (b > n) b = n;
  Fr s = Fr::zero();
  for (size_t t = b; t-- > a;) s = add(c[t], mul(z, s));
  L[j] = s;
}

// s_t for every t in chunk j, with carry-in S[j+1] (0 for the last chunk)
__global__ void __launch_bounds__(256) k_scan_chunk_final(const Fr *__restrict__ c, size_t n, Fr z,
                                                          const Fr *__restrict__ S, size_t C,
                                                          Fr *__restrict__ out) {
  size_t j = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (j >= C) return;
  size_t a = j * SCAN_K, b = a + SCAN_K;
  if (b > n) b = n;
  Fr s = (j + 1 < C) ? S[j + 1] : Fr::zero();
  for (size_t t = b; t-- > a;) {
    s = add(c[t], mul(z, s));
    out[t] = s;
  }
}

__global__ void k_scan_serial(const Fr *__restrict__ c, size_t n, Fr z, Fr *__restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  Fr s = Fr::zero();
  for (size_t t = n; t-- > 0;) {
    s = add(c[t], mul(z, s));
    out[t] = s;
  }
}

// out[t] = sum_{u >= t} c_u z^(u - t); uses scratch slots [base, base + depth)
static void suffix_scan(Ctx *ctx, const Fr *c, size_t n, const Fr &z, Fr *out, int depth) {
  if (n == 0) return;
  if (n <= (size_t)SCAN_K) {
    k_scan_serial<<<1, 64, 0, ctx->stream>>>(c, n, z, out);
    TNS_LAUNCH_CHECK();
    return;
  }
  if (depth >= 6) throw Error(TNS_ERR_POLYNOMIAL, "suffix scan too deep");
  size_t C = (n + SCAN_K - 1) / SCAN_K;
  // two arrays of C per level in one allocation
  Fr *L = (Fr *)ctx->scratch[depth].ensure(sizeof(Fr) * 2 * C);
  Fr *S = L + C;
  TNS_PROF(ctx, "open_scan", 96.0 * n);
  k_scan_chunk_local<<<grid_for(C, 256, 1u << 30), 256, 0, ctx->stream>>>(c, n, z, L, C);
  TNS_LAUNCH_CHECK();
  Fr Z = pow_u64(z, SCAN_K);
  suffix_scan(ctx, L, C, Z, S, depth + 1);
  k_scan_chunk_final<<<grid_for(C, 256, 1u << 30), 256, 0, ctx->stream>>>(c, n, z, S, C, out);
  TNS_LAUNCH_CHECK();
}

// Returns P(z); if q != nullptr, writes the n-1 quotient coefficients of
// (P - P(z)) / (x - z) there (q may alias nothing in `coeffs`).
// `s` workspace must hold n elements (ctx->scratch is used for the carries).
Fr synthetic_division_dev(Ctx *ctx, const Fr *coeffs, size_t n, const Fr &z, Fr *s) {
  if (n == 0) return Fr::zero();
  suffix_scan(ctx, coeffs, n, z, s, 0);
  Fr v;
  TNS_HIP(hipMemcpyAsync(&v, s, sizeof(Fr), hipMemcpyDeviceToHost, ctx->stream));
  TNS_HIP(hipStreamSynchronize(ctx->stream));
  return v;
}

// ---------------------------------------------------------------- conversions
__global__ void __launch_bounds__(256) k_u64_tables(const uint64_t *__restrict__ in, size_t n_in, size_t n,
                                                    Fr *__restrict__ mont, Fr *__restrict__ canon,
                                                    unsigned *__restrict__ bits) {
  unsigned b = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint64_t x = i < n_in ? in[i] : 0;
    Fr k = Fr::zero();
    k.v[0] = (uint32_t)x;
    k.v[1] = (uint32_t)(x >> 32);
    if (canon) canon[i] = k;
    mont[i] = from_u64<FrCfg>(x);
    b = x ? max(b, 64u - (unsigned)__builtin_clzll(x)) : b;
  }
  block_atomic_max2(b, 0u, bits, nullptr);
}
__global__ void __launch_bounds__(256) k_widen_u32(const uint32_t *__restrict__ in, size_t n,
                                                   uint64_t *__restrict__ out) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = in[i];
}

void widen_u32_dev(hipStream_t s, const uint32_t *in, size_t n, uint64_t *out) {
  if (!n) return;
  k_widen_u32<<<grid_for(n, 256, 4096), 256, 0, s>>>(in, n, out);
  TNS_LAUNCH_CHECK();
}

// 24-bit values packed four to three words (upload.cpp) -> u64; one thread per group of four
__global__ void __launch_bounds__(256) k_widen_u24(const uint32_t *__restrict__ in, size_t n,
                                                   uint64_t *__restrict__ out) {
  const size_t groups = (n + 3) / 4;
  for (size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x; g < groups; g += (size_t)gridDim.x * blockDim.x) {
    const uint32_t w0 = in[3 * g], w1 = in[3 * g + 1], w2 = in[3 * g + 2];
    const uint64_t v[4] = {w0 & 0xffffffu, (w0 >> 24) | ((w1 & 0xffffu) << 8), (w1 >> 16) | ((w2 & 0xffu) << 16),
                           w2 >> 8};
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (4 * g + k < n) out[4 * g + k] = v[k];
  }
}

void widen_dev(hipStream_t s, const uint32_t *in, int width, size_t n, uint64_t *out) {
  if (!n || width == 8) return;
  if (width == 4) return widen_u32_dev(s, in, n, out);
  k_widen_u24<<<grid_for((n + 3) / 4, 256, 4096), 256, 0, s>>>(in, n, out);
  TNS_LAUNCH_CHECK();
}

void u64_tables_dev(hipStream_t s, const uint64_t *in, size_t n_in, size_t n, Fr *mont, Fr *canon, unsigned *bits) {
  TNS_HIP(hipMemsetAsync(bits, 0, sizeof(unsigned), s));
  if (!n) return;
  k_u64_tables<<<grid_for(n, 256), 256, 0, s>>>(in, n_in, n, mont, canon, bits);
  TNS_LAUNCH_CHECK();
}
void fr_fill_zero_dev(Ctx *c, Fr *p, size_t n) {
  if (n) TNS_HIP(hipMemsetAsync(p, 0, n * sizeof(Fr), c->stream));
}

// ---------------------------------------------------------------- SRS generation
// setup_params (src/utils.rs:89-96): g1_powers[i] = G * tau^i, i < n.
// (1) tau^i in canonical form; (2) fixed-base comb with 32 byte-windows of
// precomputed d * 2^(8w) * G (affine, host-built table); (3) batch affine
// conversion (Montgomery's trick per chunk of points).
constexpr int SRS_POW_CHUNK = 64;

__global__ void __launch_bounds__(256) k_tau_powers(Fr tau, uint64_t e0, size_t n,
                                                    Fr *__restrict__ out_canon) {
  size_t j = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t a = j * SRS_POW_CHUNK;
  if (a >= n) return;
  size_t b = a + SRS_POW_CHUNK;
  if (b > n) b = n;
  Fr p = pow_u64(tau, e0 + (uint64_t)a);  // tau^(e0 + i)
  for (size_t i = a; i < b; i++) {
    out_canon[i] = from_mont(p);
    p = mul(p, tau);
  }
}

__global__ void __launch_bounds__(256) k_fixed_base_mul(const Fr *__restrict__ scalars_canon, size_t n,
                                                        const G1Affine *__restrict__ table,
                                                        G1Xyzz *__restrict__ out) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    Fr s = scalars_canon[i];
    G1Xyzz acc = G1Xyzz::inf();
    for (int w = 0; w < 32; w++) {
      uint32_t d = (s.v[w >> 2] >> (8 * (w & 3))) & 0xff;
      if (d) acc = xyzz_madd(acc, table[w * 256 + d]);
    }
    out[i] = acc;
  }
}

constexpr int BATCH_INV_CHUNK = 32;
// XYZZ -> affine with one inversion per chunk.  prefix: scratch of n Fq.
__global__ void __launch_bounds__(256) k_batch_to_affine(const G1Xyzz *__restrict__ in, size_t n,
                                                         Fq *__restrict__ prefix,
                                                         G1Affine *__restrict__ out) {
  size_t j = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t a = j * BATCH_INV_CHUNK;
  if (a >= n) return;
  size_t b = a + BATCH_INV_CHUNK;
  if (b > n) b = n;
  Fq acc = Fq::one();
  for (size_t i = a; i < b; i++) {
    prefix[i] = acc;
    if (!in[i].is_inf()) acc = mul(acc, in[i].zzz);
  }
  Fq iv = inv(acc);
  for (size_t i = b; i-- > a;) {
    G1Xyzz p = in[i];
    G1Affine r;
    if (p.is_inf()) {
      r.x = Fq::zero();
      r.y = Fq::zero();
    } else {
      Fq izzz = mul(iv, prefix[i]);  // 1 / ZZZ_i
      iv = mul(iv, p.zzz);
      Fq iz = mul(izzz, p.zz);  // 1 / z
      r.x = mul(p.x, sqr(iz));
      r.y = mul(p.y, izzz);
    }
    out[i] = r;
  }
}

void xyzz_to_affine_batch_dev(Ctx *c, const G1Xyzz *in, size_t n, G1Affine *out, Fq *prefix) {
  if (!n) return;
  size_t bchunks = (n + BATCH_INV_CHUNK - 1) / BATCH_INV_CHUNK;
  k_batch_to_affine<<<grid_for(bchunks, 256, 1u << 30), 256, 0, c->stream>>>(in, n, prefix, out);
  TNS_LAUNCH_CHECK();
}

// host: d * 2^(8w) * G for w < 32, d < 256 (d = 0 -> identity), affine
static std::vector<G1Affine> build_fixed_base_table() {
  std::vector<G1Xyzz> tab(32 * 256);
  G1Affine g;
  g.x = from_u64<FqCfg>(1);
  g.y = from_u64<FqCfg>(2);
  G1Xyzz base = xyzz_from_affine(g);
  for (int w = 0; w < 32; w++) {
    tab[w * 256] = G1Xyzz::inf();
    G1Xyzz acc = G1Xyzz::inf();
    for (int d = 1; d < 256; d++) {
      acc = xyzz_add(acc, base);
      tab[w * 256 + d] = acc;
    }
    for (int k = 0; k < 8; k++) base = xyzz_dbl(base);
  }
  // batch inversion of all ZZZ
  std::vector<Fq> pre(tab.size());
  Fq acc = Fq::one();
  for (size_t i = 0; i < tab.size(); i++) {
    pre[i] = acc;
    if (!tab[i].is_inf()) acc = mul(acc, tab[i].zzz);
  }
  Fq iv = inv(acc);
  std::vector<G1Affine> out(tab.size());
  for (size_t i = tab.size(); i-- > 0;) {
    if (tab[i].is_inf()) {
      out[i].x = Fq::zero();
      out[i].y = Fq::zero();
      continue;
    }
    Fq izzz = mul(iv, pre[i]);
    iv = mul(iv, tab[i].zzz);
    Fq iz = mul(izzz, tab[i].zz);
    out[i].x = mul(tab[i].x, sqr(iz));
    out[i].y = mul(tab[i].y, izzz);
  }
  return out;
}

static const G1Affine *upload_fixed_base_table(Ctx *c) {
  static std::vector<G1Affine> host_table;  // constant data; built once per process
  static std::mutex mu;
  {
    std::lock_guard<std::mutex> lk(mu);
    if (host_table.empty()) host_table = build_fixed_base_table();
  }
  G1Affine *d_table = (G1Affine *)c->scratch[0].ensure(sizeof(G1Affine) * host_table.size());
  TNS_HIP(hipMemcpyAsync(d_table, host_table.data(), sizeof(G1Affine) * host_table.size(),
                         hipMemcpyHostToDevice, c->stream));
  return d_table;
}

// out[i] = G * s_i (affine) for canonical scalars, in slabs bounding the XYZZ scratch.
// fill(off, m, dst) writes the canonical scalars of [off, off + m) into dst (device).
template <class Fill>
static void fixed_base_slabs(Ctx *c, size_t n, G1Affine *out, Fill fill) {
  if (!n) return;
  const G1Affine *d_table = upload_fixed_base_table(c);
  const size_t slab = (size_t)1 << 22;
  Fr *pw = (Fr *)c->scratch[1].ensure(sizeof(Fr) * std::min(n, slab));
  G1Xyzz *xy = (G1Xyzz *)c->scratch[2].ensure(sizeof(G1Xyzz) * std::min(n, slab));
  Fq *pre = (Fq *)c->scratch[3].ensure(sizeof(Fq) * std::min(n, slab));
  for (size_t off = 0; off < n; off += slab) {
    size_t m = std::min(slab, n - off);
    const Fr *sc = fill(off, m, pw);
    k_fixed_base_mul<<<grid_for(m, 256), 256, 0, c->stream>>>(sc, m, d_table, xy);
    TNS_LAUNCH_CHECK();
    size_t bchunks = (m + BATCH_INV_CHUNK - 1) / BATCH_INV_CHUNK;
    k_batch_to_affine<<<grid_for(bchunks, 256, 1u << 30), 256, 0, c->stream>>>(xy, m, pre, out + off);
    TNS_LAUNCH_CHECK();
  }
  TNS_HIP(hipStreamSynchronize(c->stream));
}

void srs_generate_dev(Ctx *c, const Fr &tau, size_t first, size_t n, G1Affine *out) {
  fixed_base_slabs(c, n, out, [&](size_t off, size_t m, Fr *pw) -> const Fr * {
    size_t chunks = (m + SRS_POW_CHUNK - 1) / SRS_POW_CHUNK;
    k_tau_powers<<<grid_for(chunks, 256, 1u << 30), 256, 0, c->stream>>>(tau, first + off, m, pw);
    TNS_LAUNCH_CHECK();
    return pw;
  });
}

void fixed_base_mul_dev(Ctx *c, const Fr *scalars_canon, size_t n, G1Affine *out) {
  fixed_base_slabs(c, n, out, [&](size_t off, size_t, Fr *) -> const Fr * { return scalars_canon + off; });
}

}  // namespace tns
