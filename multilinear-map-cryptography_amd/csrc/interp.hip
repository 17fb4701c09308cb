// interp.hip -- exact interpolation on the nodes {0, 1, ..., N-1} (N = 2^n) over BN254 Fr.
//
// Replaces poly_utils::lagrange_interpolate (src/polynomials.rs:301-352) as called by
// vector_to_polynomial (src/twist.rs:307-315, src/shout.rs:277-285).  The reference
// builds sum_i y_i L_i(x) in O(N^3); the interpolant's coefficients are unique, so any
// exact algorithm returns the same vector.  Ours is O(N log^2 N):
//
//  1. Newton forward differences on consecutive nodes are one convolution:
//       a_k = Delta^k y(0) / k! = sum_{j<=k} (y_j / j!) * ((-1)^(k-j) / (k-j)!)
//     so f(x) = sum_k a_k x^(k)   (x^(k) = x (x-1) ... (x-k+1), falling factorial).
//  2. Falling-factorial -> monomial by divide and conquer.  With
//       G_{s,m}(y) = sum_{k<m} a_{s+k} y^(k)
//     we have  G_{s,2m}(y) = G_{s,m}(y) + y^(m) * G_{s+m,m}(y - m).
//     y^(m) and the Taylor shift by -m depend only on m, so each level is, for every
//     block: one Taylor shift (a convolution with the fixed kernel (-m)^k/k!) and one
//     product with the fixed polynomial y^(m); both are cyclic convolutions of size 2m
//     whose fixed operand is precomputed per N (InterpPlan) in the transformed domain
//     (ntt.hip: ntt_conv_blocks, 5 HBM passes at 2m = 2^24).
// Levels whose blocks fit a 512-element LDS tile run fused in one kernel.
#include <hip/hip_runtime.h>

#include <vector>

#include "ntt.hpp"

namespace tns {

constexpr int INT_TILE_LOG = 9;  // 512-element tiles for the fused interpolation levels

__global__ void __launch_bounds__(256) k_pointwise(Fr *__restrict__ x, const Fr *__restrict__ w,
                                                   unsigned s, size_t total) {
  const size_t mask = ((size_t)1 << s) - 1;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x)
    x[i] = mul(x[i], w[i & mask]);
}
static void pointwise_blocks(Ctx *c, Fr *x, const Fr *w, unsigned s, size_t nb) {
  size_t total = nb << s;
  TNS_PROF(c, "ntt_pointwise", 96.0 * total);
  k_pointwise<<<grid_for(total, 256), 256, 0, c->stream>>>(x, w, s, total);
  TNS_LAUNCH_CHECK();
}

__global__ void __launch_bounds__(256) k_scale(Fr *__restrict__ x, Fr k, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    x[i] = mul(x[i], k);
}

// ---------------------------------------------------------------- elementwise helpers
__global__ void __launch_bounds__(256) k_iota_fr(Fr *__restrict__ out, size_t n) {  // out[i] = max(i,1)
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    out[i] = from_u64<FrCfg>(i ? i : 1);
}

// inclusive prefix product, chunked (recursive over chunk products)
constexpr int PROD_K = 64;
__global__ void k_chunk_prod(const Fr *__restrict__ in, size_t n, Fr *__restrict__ P, size_t C) {
  size_t j = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (j >= C) return;
  size_t a = j * PROD_K, b = a + PROD_K < n ? a + PROD_K : n;
  Fr p = Fr::one();
  for (size_t i = a; i < b; i++) p = mul(p, in[i]);
  P[j] = p;
}
__global__ void k_chunk_prod_final(const Fr *__restrict__ in, size_t n, const Fr *__restrict__ S,
                                   Fr *__restrict__ out, size_t C) {
  size_t j = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (j >= C) return;
  size_t a = j * PROD_K, b = a + PROD_K < n ? a + PROD_K : n;
  Fr p = j ? S[j - 1] : Fr::one();
  for (size_t i = a; i < b; i++) {
    p = mul(p, in[i]);
    out[i] = p;
  }
}
static void prefix_product(Ctx *c, const Fr *in, size_t n, Fr *out, std::vector<DevBuf *> &tmp, int depth = 0) {
  size_t C = (n + PROD_K - 1) / PROD_K;
  if (C <= 1) {
    k_chunk_prod_final<<<1, 64, 0, c->stream>>>(in, n, nullptr, out, 1);
    TNS_LAUNCH_CHECK();
    return;
  }
  if ((int)tmp.size() <= depth) tmp.push_back(new DevBuf());
  Fr *P = (Fr *)tmp[depth]->ensure(sizeof(Fr) * 2 * C);
  Fr *S = P + C;
  k_chunk_prod<<<grid_for(C, 256, 1u << 30), 256, 0, c->stream>>>(in, n, P, C);
  TNS_LAUNCH_CHECK();
  prefix_product(c, P, C, S, tmp, depth + 1);
  k_chunk_prod_final<<<grid_for(C, 256, 1u << 30), 256, 0, c->stream>>>(in, n, S, out, C);
  TNS_LAUNCH_CHECK();
}

// batch inverse (chunks of 32, one Fermat inversion each); scratch pre: n
__global__ void __launch_bounds__(256) k_batch_inverse(const Fr *__restrict__ in, size_t n,
                                                       Fr *__restrict__ pre, Fr *__restrict__ out) {
  size_t j = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t a = j * 32;
  if (a >= n) return;
  size_t b = a + 32 < n ? a + 32 : n;
  Fr acc = Fr::one();
  for (size_t i = a; i < b; i++) {
    pre[i] = acc;
    acc = mul(acc, in[i]);
  }
  Fr iv = inv(acc);
  for (size_t i = b; i-- > a;) {
    Fr x = in[i];
    out[i] = mul(iv, pre[i]);
    iv = mul(iv, x);
  }
}

// out[t] = cst^t * inv_fact[t] for t < n, zero for t in [n, len)
__global__ void __launch_bounds__(256) k_exp_series(Fr cst, const Fr *__restrict__ inv_fact, size_t n,
                                                    size_t len, Fr *__restrict__ out) {
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < len;
       t += (size_t)gridDim.x * blockDim.x)
    out[t] = t < n ? mul(pow_u64(cst, t), inv_fact[t]) : Fr::zero();
}

// ---------------------------------------------------------------- level kernels (global)
// X[b*2m + t] = t < m ? A[b*2m + m + (m-1-t)] * fact[m-1-t] : 0
__global__ void __launch_bounds__(256) k_build_u(const Fr *__restrict__ A, Fr *__restrict__ X, size_t m,
                                                 size_t total, const Fr *__restrict__ fact) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    size_t t = i & (2 * m - 1), base = i - t;
    X[i] = t < m ? mul(A[base + m + (m - 1 - t)], fact[m - 1 - t]) : Fr::zero();
  }
}
// Y[b*2m + i] = i < m ? X[b*2m + m-1-i] * inv_fact[i] : 0
__global__ void __launch_bounds__(256) k_reverse_scale(const Fr *__restrict__ X, Fr *__restrict__ Y, size_t m,
                                                       size_t total, const Fr *__restrict__ inv_fact) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    size_t t = i & (2 * m - 1), base = i - t;
    Y[i] = t < m ? mul(X[base + m - 1 - t], inv_fact[t]) : Fr::zero();
  }
}
// A[b*2m + i] = Y[b*2m + i] + (i < m ? A[b*2m + i] : 0)
__global__ void __launch_bounds__(256) k_combine(Fr *__restrict__ A, const Fr *__restrict__ Y, size_t m,
                                                 size_t total) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    size_t t = i & (2 * m - 1);
    A[i] = t < m ? add(Y[i], A[i]) : Y[i];
  }
}

// ---------------------------------------------------------------- fused low levels (LDS)
// Runs levels m = 1 .. tile/2 on tiles of `tile` coefficients of A (in place).
__global__ void __launch_bounds__(256) k_interp_tile(Fr *__restrict__ A, unsigned tile, unsigned levels,
                                                     const Fr *__restrict__ fact,
                                                     const Fr *__restrict__ inv_fact,
                                                     const Fr *__restrict__ lvl, const Fr *__restrict__ TW) {
  __shared__ Fr a[1 << INT_TILE_LOG];
  __shared__ Fr xs[1 << INT_TILE_LOG];
  Fr *g = A + (size_t)blockIdx.x * tile;
  for (unsigned i = threadIdx.x; i < tile; i += blockDim.x) a[i] = g[i];
  __syncthreads();
  for (unsigned l = 0; l < levels; l++) {
    const unsigned m = 1u << l, two_m = 2u * m;
    const Fr *Vhat = lvl + 4 * ((size_t)m - 1);
    const Fr *Phat = Vhat + two_m;
    for (unsigned i = threadIdx.x; i < tile; i += blockDim.x) {
      unsigned t = i & (two_m - 1), base = i - t;
      xs[i] = t < m ? mul(a[base + m + (m - 1 - t)], fact[m - 1 - t]) : Fr::zero();
    }
    __syncthreads();
    lds_ntt<false>(xs, tile, (int)l, TW);
    for (unsigned i = threadIdx.x; i < tile; i += blockDim.x) xs[i] = mul(xs[i], Vhat[i & (two_m - 1)]);
    __syncthreads();
    lds_ntt<true>(xs, tile, (int)l, TW);
    // reversal + 1/i! (read all, then write)
    Fr tmp[(1 << INT_TILE_LOG) / 256];
    {
      int q = 0;
      for (unsigned i = threadIdx.x; i < tile; i += blockDim.x, q++) {
        unsigned t = i & (two_m - 1), base = i - t;
        tmp[q] = t < m ? mul(xs[base + m - 1 - t], inv_fact[t]) : Fr::zero();
      }
    }
    __syncthreads();
    {
      int q = 0;
      for (unsigned i = threadIdx.x; i < tile; i += blockDim.x, q++) xs[i] = tmp[q];
    }
    __syncthreads();
    lds_ntt<false>(xs, tile, (int)l, TW);
    for (unsigned i = threadIdx.x; i < tile; i += blockDim.x) xs[i] = mul(xs[i], Phat[i & (two_m - 1)]);
    __syncthreads();
    lds_ntt<true>(xs, tile, (int)l, TW);
    for (unsigned i = threadIdx.x; i < tile; i += blockDim.x) {
      unsigned t = i & (two_m - 1);
      a[i] = t < m ? add(xs[i], a[i]) : xs[i];
    }
    __syncthreads();
  }
  for (unsigned i = threadIdx.x; i < tile; i += blockDim.x) g[i] = a[i];
}

// ---------------------------------------------------------------- plan construction
__global__ void k_copy_fr(const Fr *__restrict__ in, Fr *__restrict__ out, size_t n, size_t len) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < len;
       i += (size_t)gridDim.x * blockDim.x)
    out[i] = i < n ? in[i] : Fr::zero();
}
// out[i] = C(m, i) (-m)^(m-i), i <= m  (the binomial expansion of (y - m)^m)
__global__ void k_binom_shift(size_t m, Fr negm, const Fr *__restrict__ fact, const Fr *__restrict__ inv_fact,
                              Fr *__restrict__ out) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i <= m; i += (size_t)gridDim.x * blockDim.x)
    out[i] = mul(mul(mul(fact[m], inv_fact[i]), inv_fact[m - i]), pow_u64(negm, m - i));
}
__global__ void k_add_into(Fr *__restrict__ a, const Fr *__restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = add(a[i], b[i]);
}

// fact[k] = k!, ifact[k] = 1/k! for k < nf (device; synchronises the stream)
void factorial_tables_dev(Ctx *c, size_t nf, Fr *fact, Fr *ifact) {
  hipStream_t st = c->stream;
  DevBuf iota, pre;
  Fr *io = (Fr *)iota.ensure(sizeof(Fr) * nf);
  k_iota_fr<<<grid_for(nf, 256), 256, 0, st>>>(io, nf);
  TNS_LAUNCH_CHECK();
  std::vector<DevBuf *> tmp;
  prefix_product(c, io, nf, fact, tmp);
  Fr *pr = (Fr *)pre.ensure(sizeof(Fr) * nf);
  k_batch_inverse<<<grid_for((nf + 31) / 32, 256, 1u << 30), 256, 0, st>>>(fact, nf, pr, ifact);
  TNS_LAUNCH_CHECK();
  TNS_HIP(hipStreamSynchronize(st));
  for (auto *b : tmp) delete b;
}

static Fr fr_inv_pow2(unsigned s) { return inv(from_u64<FrCfg>((uint64_t)1 << s)); }

// forward transform of `len` coefficients zero-padded to 2^s, scaled by 2^-s (a conv operand)
static void make_conv_operand(Ctx *c, const Fr *coeffs, size_t len, unsigned s, Fr *out) {
  const size_t S = (size_t)1 << s;
  k_copy_fr<<<grid_for(S, 256), 256, 0, c->stream>>>(coeffs, out, len, S);
  TNS_LAUNCH_CHECK();
  ntt_blocks(c, out, s, 1, false);
  k_scale<<<grid_for(S, 256), 256, 0, c->stream>>>(out, fr_inv_pow2(s), S);
  TNS_LAUNCH_CHECK();
}

static InterpPlan *get_plan(Ctx *c, unsigned log_n) {
  if (c->plans.size() <= log_n) c->plans.resize(log_n + 1, nullptr);
  if (c->plans[log_n]) return c->plans[log_n];
  const size_t N = (size_t)1 << log_n;
  const size_t NF = N < 4 ? 4 : N;  // factorial table length (>= m + 1 for every level)
  InterpPlan *P = new InterpPlan();
  P->log_n = log_n;
  ntt_twiddles(c, log_n + 2);
  hipStream_t st = c->stream;
  // factorials
  Fr *fact = (Fr *)P->fact.ensure(sizeof(Fr) * NF);
  Fr *ifact = (Fr *)P->inv_fact.ensure(sizeof(Fr) * NF);
  factorial_tables_dev(c, NF, fact, ifact);
  // Newton kernel: NTT_{2N}((-1)^t / t!) / (2N)
  {
    Fr *wh = (Fr *)P->newton_kernel_hat.ensure(sizeof(Fr) * 2 * N);
    k_exp_series<<<grid_for(2 * N, 256), 256, 0, st>>>(neg(Fr::one()), ifact, N, 2 * N, wh);
    TNS_LAUNCH_CHECK();
    ntt_blocks(c, wh, log_n + 1, 1, false);
    k_scale<<<grid_for(2 * N, 256), 256, 0, st>>>(wh, fr_inv_pow2(log_n + 1), 2 * N);
    TNS_LAUNCH_CHECK();
  }
  // per-level tables: level l (m = 2^l) at offset 4(m - 1): Vhat (2m) | Phat (2m)
  if (log_n >= 1) {
    Fr *lv = (Fr *)P->level_tables.ensure(sizeof(Fr) * 4 * N);
    DevBuf pm_b, q_b, t1_b, t2_b;
    Fr *pm = (Fr *)pm_b.ensure(sizeof(Fr) * 2 * N);  // coefficients of y^(m) (m+1 used)
    Fr *q = (Fr *)q_b.ensure(sizeof(Fr) * 2 * N);
    Fr *t1 = (Fr *)t1_b.ensure(sizeof(Fr) * 2 * N);
    Fr *t2 = (Fr *)t2_b.ensure(sizeof(Fr) * 2 * N);
    {
      Fr h[2] = {Fr::zero(), Fr::one()};  // y^(1) = y
      TNS_HIP(hipMemcpyAsync(pm, h, sizeof h, hipMemcpyHostToDevice, st));
    }
    for (unsigned l = 0; l < log_n; l++) {
      const size_t m = (size_t)1 << l;
      Fr *Vhat = lv + 4 * (m - 1), *Phat = Vhat + 2 * m;
      const Fr negm = neg(from_u64<FrCfg>(m));
      // Vhat: NTT_{2m}((-m)^k / k!, k < m) / 2m
      k_exp_series<<<grid_for(2 * m, 256), 256, 0, st>>>(negm, ifact, m, 2 * m, t1);
      TNS_LAUNCH_CHECK();
      make_conv_operand(c, t1, 2 * m, l + 1, Vhat);
      // Phat: NTT_{2m}(y^(m)) / 2m  (m+1 coefficients, padded)
      make_conv_operand(c, pm, m + 1, l + 1, Phat);
      if (l + 1 == log_n) break;
      // y^(2m) = y^(m) * (y-m)^(m);  (y-m)^(m) = (y-m)^m + p(y - m) with p = y^(m) - y^m.
      // Taylor shift of p (m coefficients) by -m as a size-4m convolution.
      const unsigned s4 = l + 2;
      const size_t L4 = (size_t)4 * m;
      k_copy_fr<<<grid_for(L4, 256), 256, 0, st>>>(pm, t2, m, L4);  // t2 = p
      TNS_LAUNCH_CHECK();
      k_build_u<<<grid_for(2 * m, 256), 256, 0, st>>>(t2 - m, t1, m, 2 * m, fact);  // t1 = rev(p) * k!
      TNS_LAUNCH_CHECK();
      k_copy_fr<<<grid_for(L4 - 2 * m, 256), 256, 0, st>>>(t1, t1 + 2 * m, 0, L4 - 2 * m);  // zero tail
      TNS_LAUNCH_CHECK();
      k_exp_series<<<grid_for(L4, 256), 256, 0, st>>>(negm, ifact, m, L4, t2);
      TNS_LAUNCH_CHECK();
      make_conv_operand(c, t2, L4, s4, q);  // q: transformed kernel (scratch)
      ntt_conv_blocks(c, t1, s4, 1, q);
      // q[i] = t1[m-1-i] / i!  (i < m) -> p(y - m);  plus the binomial part for i <= m
      k_reverse_scale<<<grid_for(2 * m, 256), 256, 0, st>>>(t1, q, m, 2 * m, ifact);
      TNS_LAUNCH_CHECK();
      k_binom_shift<<<grid_for(m + 1, 256), 256, 0, st>>>(m, negm, fact, ifact, t2);
      TNS_LAUNCH_CHECK();
      k_add_into<<<grid_for(m + 1, 256), 256, 0, st>>>(q, t2, m + 1);
      TNS_LAUNCH_CHECK();
      // y^(2m) = pm * q   (both m+1 coefficients; product 2m+1 <= 4m)
      make_conv_operand(c, q, m + 1, s4, t2);
      k_copy_fr<<<grid_for(L4, 256), 256, 0, st>>>(pm, t1, m + 1, L4);
      TNS_LAUNCH_CHECK();
      ntt_conv_blocks(c, t1, s4, 1, t2);
      k_copy_fr<<<grid_for(2 * m + 1, 256), 256, 0, st>>>(t1, pm, 2 * m + 1, 2 * m + 1);
      TNS_LAUNCH_CHECK();
    }
    TNS_HIP(hipStreamSynchronize(st));
  }
  c->plans[log_n] = P;
  return P;
}

// ---------------------------------------------------------------- entry point
// coeffs (device, n) <- interpolant of y (device, n) on nodes 0..n-1, n a power of two
// (Twist/Shout always pad to powers of two before interpolating, src/twist.rs:141-152).
void interpolate_consecutive_dev(Ctx *c, const Fr *y, size_t n, Fr *coeffs) {
  if (n == 0) return;
  if (n & (n - 1)) throw Error(TNS_ERR_POLYNOMIAL, "interpolation size must be a power of two");
  const unsigned log_n = ilog2_exact(n);
  hipStream_t st = c->stream;
  if (n == 1) {
    TNS_HIP(hipMemcpyAsync(coeffs, y, sizeof(Fr), hipMemcpyDeviceToDevice, st));
    return;
  }
  InterpPlan *P = get_plan(c, log_n);
  const Fr *fact = P->fact.as<Fr>(), *ifact = P->inv_fact.as<Fr>();
  Fr *X2 = (Fr *)c->scratch[6].ensure(sizeof(Fr) * 2 * n);
  Fr *A = coeffs;
  // 1. Newton coefficients: first n entries of conv(y_j / j!, (-1)^t / t!)
  {
    TNS_PROF(c, "interp_elementwise", 64.0 * 2 * n);
    k_copy_fr<<<grid_for(2 * n, 256), 256, 0, st>>>(y, X2, n, 2 * n);
    TNS_LAUNCH_CHECK();
  }
  pointwise_blocks(c, X2, ifact, log_n, 1);  // first n entries *= 1/j!
  ntt_conv_blocks(c, X2, log_n + 1, 1, P->newton_kernel_hat.as<Fr>());
  TNS_HIP(hipMemcpyAsync(A, X2, sizeof(Fr) * n, hipMemcpyDeviceToDevice, st));
  // 2. levels
  const Fr *lv = P->level_tables.as<Fr>();
  const Fr *TW = ntt_twiddles(c, log_n + 2);
  const unsigned tile_log = log_n < INT_TILE_LOG ? log_n : INT_TILE_LOG;
  const unsigned tile = 1u << tile_log;
  {
    TNS_PROF(c, "interp_tile", 64.0 * n);
    k_interp_tile<<<(unsigned)(n / tile), 256, 0, st>>>(A, tile, tile_log, fact, ifact, lv, TW);
    TNS_LAUNCH_CHECK();
  }
  Fr *X = X2, *Y = X2 + n;
  for (unsigned l = tile_log; l < log_n; l++) {
    const size_t m = (size_t)1 << l;
    const size_t nb = n / (2 * m);
    const Fr *Vhat = lv + 4 * (m - 1), *Phat = Vhat + 2 * m;
    {
      TNS_PROF(c, "interp_elementwise", 64.0 * n);
      k_build_u<<<grid_for(n, 256), 256, 0, st>>>(A, X, m, n, fact);
      TNS_LAUNCH_CHECK();
    }
    ntt_conv_blocks(c, X, l + 1, nb, Vhat);  // Taylor shift by -m
    {
      TNS_PROF(c, "interp_elementwise", 64.0 * n);
      k_reverse_scale<<<grid_for(n, 256), 256, 0, st>>>(X, Y, m, n, ifact);
      TNS_LAUNCH_CHECK();
    }
    ntt_conv_blocks(c, Y, l + 1, nb, Phat);  // times y^(m)
    {
      TNS_PROF(c, "interp_elementwise", 96.0 * n);
      k_combine<<<grid_for(n, 256), 256, 0, st>>>(A, Y, m, n);
      TNS_LAUNCH_CHECK();
    }
  }
}

}  // namespace tns
