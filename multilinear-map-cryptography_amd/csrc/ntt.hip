// ntt.hip -- radix-2 NTT engine over BN254 Fr, organised around HBM passes.
//
// A transform of size 2^s over nb contiguous blocks runs as
//   * strided LDS passes for the large strides: a 256-thread workgroup stages a
//     2^r x 32 tile (rows 2^lo apart, 32 consecutive columns = 1 KiB contiguous per
//     row, so each row is a whole DRAM burst run and page) and runs r <= 5 stages in
//     LDS before writing back -- one HBM read and write per r stages instead of per stage;
//   * a contiguous 1024-element LDS tile for the 10 smallest strides.
// ntt_conv_blocks fuses the last forward tile pass, the pointwise product and the
// first inverse tile pass into one kernel, so a size-2^24 cyclic convolution is
// 2 + 1 + 2 = 5 passes over HBM.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "ntt.hpp"

namespace tns {

constexpr int TILE_LOG = 10;   // contiguous LDS tile: 1024 Fr = 32 KiB
constexpr int PASS_COLS = 32;  // columns per strided tile: 1 KiB contiguous per row (page/TLB friendly)
constexpr int PASS_RMAX = 5;   // stages per strided pass: 2^5 rows x 32 cols = 1024 Fr

// Fr two-adic root of unity of order 2^28 (= 5^((r-1)/2^28); ark-bn254 TWO_ADIC_ROOT_OF_UNITY)
Fr fr_root_of_unity(unsigned log_order) {
  const uint32_t c[8] = {0x725b19f0u, 0x9bd61b6eu, 0x41112ed4u, 0x402d111eu,
                         0x8ef62abcu, 0x00e0a7ebu, 0xa58a7e85u, 0x2a3c09f0u};
  Fr x;
  for (int i = 0; i < 8; i++) x.v[i] = c[i];
  x = to_mont(x);
  for (unsigned i = log_order; i < 28; i++) x = sqr(x);
  return x;
}

struct StageRoots {
  Fr w[29];  // w[lh] = primitive 2^(lh+1)-th root (the root of a size-2h stage)
};

// TW[i] for i in [1, n): stage lh = floor(log2 i), k = i - 2^lh, TW[i] = w_{2^(lh+1)}^k
__global__ void __launch_bounds__(256) k_stage_twiddles(StageRoots R, size_t n, Fr *__restrict__ TW) {
  size_t j = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t a = j * 64;
  if (a >= n) return;
  size_t b = a + 64 < n ? a + 64 : n;
  if (a == 0) {
    TW[0] = Fr::one();
    a = 1;
  }
  Fr p = Fr::one(), w = Fr::one();
  int cur_lh = -1;
  for (size_t i = a; i < b; i++) {
    int lh = 63 - __builtin_clzll((unsigned long long)i);
    size_t k = i - ((size_t)1 << lh);
    if (lh != cur_lh) {
      cur_lh = lh;
      w = R.w[lh];
      p = pow_u64(w, k);
    }
    TW[i] = p;
    p = mul(p, w);
  }
}

const Fr *ntt_twiddles(Ctx *c, unsigned L) {
  if (L < 1) L = 1;
  if (c->twiddle_log >= L) return c->twiddles.as<Fr>();
  if (L > 28) throw Error(TNS_ERR_POLYNOMIAL, "NTT larger than 2^28 (Fr two-adicity)");
  StageRoots R;
  for (unsigned lh = 0; lh < 28; lh++) R.w[lh] = fr_root_of_unity(lh + 1);
  R.w[28] = Fr::one();
  const size_t n = (size_t)1 << L;
  Fr *tw = (Fr *)c->twiddles.ensure(sizeof(Fr) * n);
  k_stage_twiddles<<<grid_for((n + 63) / 64, 256, 1u << 30), 256, 0, c->stream>>>(R, n, tw);
  TNS_LAUNCH_CHECK();
  c->twiddle_log = L;
  return tw;
}

// ---------------------------------------------------------------- contiguous LDS tiles
template <bool INV>
__global__ void __launch_bounds__(256) k_ntt_tile(Fr *__restrict__ x, unsigned tile, int lh_hi,
                                                  const Fr *__restrict__ TW) {
  __shared__ Fr buf[1 << TILE_LOG];
  Fr *base = x + (size_t)blockIdx.x * tile;
  for (unsigned i = threadIdx.x; i < tile; i += blockDim.x) buf[i] = base[i];
  __syncthreads();
  lds_ntt<INV>(buf, tile, lh_hi, TW);
  for (unsigned i = threadIdx.x; i < tile; i += blockDim.x) base[i] = buf[i];
}

// forward low stages -> multiply by w[(global index) & wmask] -> inverse low stages
__global__ void __launch_bounds__(256) k_ntt_tile_conv(Fr *__restrict__ x, unsigned tile, int lh_hi,
                                                       const Fr *__restrict__ w, size_t wmask,
                                                       const Fr *__restrict__ TW) {
  __shared__ Fr buf[1 << TILE_LOG];
  const size_t g0 = (size_t)blockIdx.x * tile;
  Fr *base = x + g0;
  for (unsigned i = threadIdx.x; i < tile; i += blockDim.x) buf[i] = base[i];
  __syncthreads();
  lds_ntt<false>(buf, tile, lh_hi, TW);
  for (unsigned i = threadIdx.x; i < tile; i += blockDim.x) buf[i] = mul(buf[i], w[(g0 + i) & wmask]);
  __syncthreads();
  lds_ntt<true>(buf, tile, lh_hi, TW);
  for (unsigned i = threadIdx.x; i < tile; i += blockDim.x) base[i] = buf[i];
}

// ---------------------------------------------------------------- strided multi-stage pass
// Stages lh in [lo, lo + r) of super-blocks of M = 2^(lo+r) elements, on tiles of 2^r rows
// (2^lo apart) x PASS_COLS consecutive columns, in four-step form: the stages' twiddle
// w_{2h}^{(j mod 2^ll) 2^lo + c} factors into a size-2^r sub-DFT twiddle (tiny table) and
// a column term that commutes to one multiply per element by w_M^{c rev_r(j)}
// (forward: after the sub-DFT; inverse: w_M^{-c rev_r(j)} before it).  The per-pass
// table PT[j 2^lo + c] has the data's own layout, so it streams coalesced with the tile.
__global__ void __launch_bounds__(256) k_pass_twiddles(const Fr *__restrict__ TW, unsigned lo, unsigned r,
                                                       Fr *__restrict__ fwd, Fr *__restrict__ inv_) {
  const size_t M = (size_t)1 << (lo + r), half = M >> 1;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < M; i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t j = (uint32_t)(i >> lo), c = (uint32_t)(i & (((size_t)1 << lo) - 1));
    const uint32_t rj = __brev(j) >> (32 - r);
    const size_t e = (size_t)c * rj;  // < M
    auto pw = [&](size_t ex) { return ex < half ? TW[half + ex] : neg(TW[ex]); };  // w_M^ex
    fwd[i] = pw(e);
    inv_[i] = e ? pw(M - e) : Fr::one();
  }
}

static const Fr *pass_table(Ctx *c, unsigned lo, unsigned r) {
  const uint32_t key = (lo << 8) | r;
  auto it = c->pass_tw.find(key);
  if (it != c->pass_tw.end()) return it->second->as<Fr>();
  const Fr *TW = ntt_twiddles(c, lo + r);
  const size_t M = (size_t)1 << (lo + r);
  DevBuf *b = new DevBuf();
  Fr *t = (Fr *)b->ensure(sizeof(Fr) * 2 * M);
  k_pass_twiddles<<<grid_for(M, 256), 256, 0, c->stream>>>(TW, lo, r, t, t + M);
  TNS_LAUNCH_CHECK();
  c->pass_tw[key] = b;
  return t;
}

template <bool INV>
__global__ void __launch_bounds__(256) k_ntt_pass(Fr *__restrict__ x, size_t ntiles, unsigned lo, unsigned r,
                                                  const Fr *__restrict__ PT, const Fr *__restrict__ TW) {
  __shared__ Fr buf[(1 << PASS_RMAX) * PASS_COLS];
  constexpr int PER = ((1 << PASS_RMAX) * PASS_COLS) / 256;
  const unsigned rows = 1u << r, elems = rows * PASS_COLS;
  const size_t cgroups = ((size_t)1 << lo) / PASS_COLS;
  for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const size_t outer = t / cgroups, cg = t % cgroups;
    const size_t base = (outer << (lo + r)) + cg * PASS_COLS;
    Fr tw[PER];
#pragma unroll
    for (int q = 0; q < PER; q++) {
      const unsigned e = threadIdx.x + 256 * q;
      if (e < elems) {
        const size_t off = ((size_t)(e / PASS_COLS) << lo) + cg * PASS_COLS + (e % PASS_COLS);
        tw[q] = PT[off];
        Fr v = x[(outer << (lo + r)) + off];
        buf[e] = INV ? mul(v, tw[q]) : v;
      }
    }
    __syncthreads();
    lds_stages<INV, PASS_COLS, true>(buf, rows, (int)r - 1, 0, 0, TW);
#pragma unroll
    for (int q = 0; q < PER; q++) {
      const unsigned e = threadIdx.x + 256 * q;
      if (e < elems) {
        Fr v = buf[e];
        x[base + ((size_t)(e / PASS_COLS) << lo) + (e % PASS_COLS)] = INV ? v : mul(v, tw[q]);
      }
    }
    __syncthreads();
  }
}

// stages [T, s) split into passes of <= PASS_RMAX stages; DIF runs them high -> low
static void strided_passes(Ctx *c, Fr *x, unsigned s, unsigned T, size_t total, bool inverse, const Fr *TW) {
  if (s <= T) return;
  const unsigned R = s - T;
  const unsigned np = (R + PASS_RMAX - 1) / PASS_RMAX;
  std::vector<std::pair<unsigned, unsigned>> passes;  // (lo, r), low to high
  unsigned lo = T;
  for (unsigned p = 0; p < np; p++) {
    unsigned r = R / np + (p < R % np ? 1 : 0);
    passes.push_back({lo, r});
    lo += r;
  }
  if (!inverse) std::reverse(passes.begin(), passes.end());
  for (auto &pr : passes) {
    const Fr *PT = pass_table(c, pr.first, pr.second);
    const size_t M = (size_t)1 << (pr.first + pr.second);
    const size_t ntiles = total >> (pr.second + 5);  // 2^r rows x 32 cols per tile
    const unsigned grid = (unsigned)std::min<size_t>(ntiles, 8192);
    TNS_PROF(c, "ntt_stage", 64.0 * total);
    if (!inverse)
      k_ntt_pass<false><<<grid, 256, 0, c->stream>>>(x, ntiles, pr.first, pr.second, PT, TW);
    else
      k_ntt_pass<true><<<grid, 256, 0, c->stream>>>(x, ntiles, pr.first, pr.second, PT + M, TW);
    TNS_LAUNCH_CHECK();
  }
}

void ntt_blocks(Ctx *c, Fr *x, unsigned s, size_t nb, bool inverse) {
  if (s == 0) return;
  const Fr *TW = ntt_twiddles(c, s);
  const size_t total = nb << s;
  const unsigned T = s < (unsigned)TILE_LOG ? s : (unsigned)TILE_LOG;
  size_t tile = (size_t)1 << T;
  const size_t ntiles = total / tile;
  if (!inverse) {
    strided_passes(c, x, s, T, total, false, TW);
    TNS_PROF(c, "ntt_lds", 64.0 * total);
    k_ntt_tile<false><<<(unsigned)ntiles, 256, 0, c->stream>>>(x, (unsigned)tile, (int)T - 1, TW);
    TNS_LAUNCH_CHECK();
  } else {
    {
      TNS_PROF(c, "ntt_lds", 64.0 * total);
      k_ntt_tile<true><<<(unsigned)ntiles, 256, 0, c->stream>>>(x, (unsigned)tile, (int)T - 1, TW);
      TNS_LAUNCH_CHECK();
    }
    strided_passes(c, x, s, T, total, true, TW);
  }
}

void ntt_conv_blocks(Ctx *c, Fr *x, unsigned s, size_t nb, const Fr *w) {
  if (s == 0) {
    throw Error(TNS_ERR_POLYNOMIAL, "ntt_conv_blocks: empty transform");
  }
  const Fr *TW = ntt_twiddles(c, s);
  const size_t total = nb << s;
  const unsigned T = s < (unsigned)TILE_LOG ? s : (unsigned)TILE_LOG;
  const size_t tile = (size_t)1 << T;
  strided_passes(c, x, s, T, total, false, TW);
  {
    TNS_PROF(c, "ntt_lds", 96.0 * total);
    k_ntt_tile_conv<<<(unsigned)(total / tile), 256, 0, c->stream>>>(x, (unsigned)tile, (int)T - 1, w,
                                                                     ((size_t)1 << s) - 1, TW);
    TNS_LAUNCH_CHECK();
  }
  strided_passes(c, x, s, T, total, true, TW);
}

}  // namespace tns
