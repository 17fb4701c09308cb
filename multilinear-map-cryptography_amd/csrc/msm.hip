// msm.hip -- BN254 G1 multi-scalar multiplication (Pippenger, signed windows).
//
// Replaces KZGCommitment::commit's per-term scalar multiplications
// (src/commitments.rs:173-177): C = sum_i c_i * g1_powers[i].  The group element
// is unique, so any correct algorithm reproduces it exactly.
//
// Pipeline (all on one stream):
//  1. k_digits: scalar -> canonical -> W signed c-bit digits; key = (window, |d|-1),
//     value = point index | sign<<31; zero digits get a sentinel key.
//  2. rocPRIM/hipCUB radix sort of the W*n (key, value) pairs by key.
//  3. k_bucket_bounds: [start, end) of every bucket in the sorted order.
//  4. k_accumulate: load-balanced -- each thread owns K consecutive sorted entries
//     and XYZZ-madds the (possibly negated) affine points run by run; runs that
//     cross a chunk boundary leave a head/tail partial.
//  5. k_bucket_fixup: buckets spanning chunks = tail + heads; empty -> identity.
//  6. k_bucket_reduce + k_window_sum: S_w = sum_j (j+1) B_{w,j} via per-group
//     running sums, then a block tree per window.
//  7. host: sum_w 2^(c w) S_w (Horner, W*c doublings).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <vector>

#include "common.hpp"

namespace tns {

constexpr int ACC_K = 32;      // sorted entries per accumulation thread
constexpr int RED_L = 16;      // buckets per reduction thread

struct MsmPlan {
  int c, W, wbits;
  uint32_t sentinel;
  int end_bit;
  size_t nb;  // W * 2^(c-1)
};

// bits: bit length of the largest scalar (the windows above it are all zero; commitments
// to traces -- addresses, small values, flags -- often have bits << 254)
static MsmPlan make_plan(size_t n, int bits) {
  MsmPlan p;
  int lg = 0;
  while (((size_t)1 << lg) < n) lg++;
  // the top window must not produce a carry: its raw value < 2^(bits - c(W-1)) must be <= 2^(c-1)
  auto windows = [bits](int c) {
    int W = (bits + c - 1) / c;
    if (bits - c * (W - 1) > c - 1) W++;
    return W;
  };
  // window c minimising (bucket adds) W*n + (reduction adds) ~3*W*2^(c-1)
  double best = 1e300;
  p.c = 4;
  for (int c = 4; c <= 20 && c <= lg + 1; c++) {
    double cost = (double)windows(c) * (double)n + 3.0 * windows(c) * (double)(1u << (c - 1));
    if (cost < best * 0.98) {  // prefer the smaller window on near-ties (less bucket memory)
      best = cost;
      p.c = c;
    }
  }
  p.W = windows(p.c);
  p.wbits = 0;
  while ((1 << p.wbits) < p.W) p.wbits++;
  p.end_bit = p.wbits + (p.c - 1) + 1;
  p.sentinel = 1u << (p.wbits + p.c - 1);
  p.nb = (size_t)p.W << (p.c - 1);
  return p;
}

// *bits = max over i of bitlen(canonical scalar_i)
__global__ void __launch_bounds__(256) k_scalar_bits(const Fr *__restrict__ scalars, size_t n,
                                                     unsigned *__restrict__ bits) {
  unsigned b = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    Fr k = from_mont(scalars[i]);
    for (int l = 7; l >= 0; l--)
      if (k.v[l]) {
        unsigned bl = 32 * l + 32 - __builtin_clz(k.v[l]);
        b = bl > b ? bl : b;
        break;
      }
  }
  for (int o = 32; o > 0; o >>= 1) {
    unsigned x = __shfl_xor(b, o);
    b = x > b ? x : b;
  }
  if ((threadIdx.x & 63) == 0 && b) atomicMax(bits, b);
}

__global__ void __launch_bounds__(256) k_digits(const Fr *__restrict__ scalars, size_t n, int c, int W,
                                                uint32_t sentinel, uint32_t *__restrict__ keys,
                                                uint32_t *__restrict__ vals) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    Fr k = from_mont(scalars[i]);
    uint32_t carry = 0;
    const uint32_t half = 1u << (c - 1);
    for (int w = 0; w < W; w++) {
      int bit = w * c;
      int limb = bit >> 5, sh = bit & 31;
      uint64_t lo = limb < 8 ? k.v[limb] : 0;
      uint64_t hi = limb + 1 < 8 ? k.v[limb + 1] : 0;
      uint32_t raw = (uint32_t)(((lo | (hi << 32)) >> sh) & ((1u << c) - 1));
      uint32_t val = raw + carry;
      uint32_t key, neg = 0, mag;
      if (val > half) {
        mag = (1u << c) - val;
        neg = 1;
        carry = 1;
      } else {
        mag = val;
        carry = 0;
      }
      key = mag ? (((uint32_t)w << (c - 1)) | (mag - 1)) : sentinel;
      keys[(size_t)w * n + i] = key;
      vals[(size_t)w * n + i] = (uint32_t)i | (neg << 31);
    }
  }
}

__global__ void __launch_bounds__(256) k_bucket_bounds(const uint32_t *__restrict__ keys, size_t total,
                                                       uint32_t sentinel, uint32_t *__restrict__ start,
                                                       uint32_t *__restrict__ end,
                                                       uint32_t *__restrict__ valid) {
  for (size_t p = blockIdx.x * (size_t)blockDim.x + threadIdx.x; p < total;
       p += (size_t)gridDim.x * blockDim.x) {
    uint32_t k = keys[p];
    if (k == sentinel) continue;
    if (p == 0 || keys[p - 1] != k) start[k] = (uint32_t)p;
    uint32_t nx = (p + 1 < total) ? keys[p + 1] : sentinel;
    if (nx != k) end[k] = (uint32_t)(p + 1);
    if (nx == sentinel) *valid = (uint32_t)(p + 1);
  }
}

struct HeadTail {
  G1Xyzz head, tail;
};

__device__ __forceinline__ G1Affine load_signed_point(const G1Affine *__restrict__ pts, uint32_t v) {
  G1Affine p = pts[v & 0x7fffffffu];
  if (v >> 31) p.y = neg(p.y);
  return p;
}

__global__ void __launch_bounds__(256) k_accumulate(const uint32_t *__restrict__ keys,
                                                    const uint32_t *__restrict__ vals,
                                                    const uint32_t *__restrict__ valid_p,
                                                    const uint32_t *__restrict__ start,
                                                    const uint32_t *__restrict__ end,
                                                    const G1Affine *__restrict__ pts,
                                                    G1Xyzz *__restrict__ buckets,
                                                    HeadTail *__restrict__ ht, size_t nchunks) {
  const size_t valid = *valid_p;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < nchunks;
       t += (size_t)gridDim.x * blockDim.x) {
    const size_t a = t * ACC_K;
    if (a >= valid) continue;
    size_t b = a + ACC_K;
    if (b > valid) b = valid;
    uint32_t cur = keys[a];
    G1Xyzz acc = G1Xyzz::inf();
    for (size_t p = a;; p++) {
      uint32_t k = (p < b) ? keys[p] : 0xffffffffu;
      if (k != cur) {
        // flush run of bucket `cur`
        uint32_t s = start[cur], e = end[cur];
        if (s < a) ht[t].head = acc;
        else if (e > b) ht[t].tail = acc;
        else buckets[cur] = acc;
        if (p >= b) break;
        cur = k;
        acc = G1Xyzz::inf();
      }
      acc = xyzz_madd(acc, load_signed_point(pts, vals[p]));
    }
  }
}

// Heavy buckets (skewed scalars: repeated values, small ranges) span many chunks; their
// chunk heads are summed through a 32-ary hierarchy so no thread walks a long run.
// Level l >= 1, group g covers chunks [g 32^l, (g+1) 32^l); its sum is formed only when
// every sorted entry of those chunks has one key (then every head in it is a full-chunk
// sum of that bucket); other groups are never read by the fixup below.
constexpr int FIX_FAN = 32;
constexpr int FIX_LEVELS = 5;
struct FixLevels {
  G1Xyzz *lv[FIX_LEVELS + 1];  // lv[l] for l >= 1 (lv[0] unused: the heads live in ht)
  size_t len[FIX_LEVELS + 1];
  int n;                        // levels built (0: none)
};

__global__ void __launch_bounds__(256) k_fix_level(const uint32_t *__restrict__ keys,
                                                   const uint32_t *__restrict__ valid_p,
                                                   const HeadTail *__restrict__ ht, const G1Xyzz *__restrict__ below,
                                                   int level, size_t n_groups, G1Xyzz *__restrict__ out) {
  const size_t valid = *valid_p;
  for (size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x; g < n_groups; g += (size_t)gridDim.x * blockDim.x) {
    size_t span = (size_t)ACC_K;
    for (int l = 0; l < level; l++) span *= FIX_FAN;
    const size_t a = g * span, b = a + span;  // entries covered
    if (b > valid || keys[a] != keys[b - 1]) continue;
    G1Xyzz acc = level == 1 ? ht[g * FIX_FAN].head : below[g * FIX_FAN];
    for (int i = 1; i < FIX_FAN; i++)
      acc = xyzz_add(acc, level == 1 ? ht[g * FIX_FAN + i].head : below[g * FIX_FAN + i]);
    out[g] = acc;
  }
}

__global__ void __launch_bounds__(256) k_bucket_fixup(const uint32_t *__restrict__ start,
                                                      const uint32_t *__restrict__ end,
                                                      const HeadTail *__restrict__ ht, FixLevels F,
                                                      G1Xyzz *__restrict__ buckets, size_t nb) {
  for (size_t bk = blockIdx.x * (size_t)blockDim.x + threadIdx.x; bk < nb;
       bk += (size_t)gridDim.x * blockDim.x) {
    uint32_t s = start[bk], e = end[bk];
    if (s == e) {
      buckets[bk] = G1Xyzz::inf();
      continue;
    }
    size_t tf = s / ACC_K, tl = (e - 1) / ACC_K;
    if (tf == tl) continue;
    G1Xyzz acc = xyzz_add(ht[tf].tail, ht[tl].head);
    // heads of the chunks strictly inside (tf, tl) -- single-key chunks: peel to
    // FIX_FAN-aligned ranges, then climb a level
    size_t lo = tf + 1, hi = tl;
    int l = 0;
    for (;;) {
      auto at = [&](size_t i) { return l == 0 ? ht[i].head : F.lv[l][i]; };
      if (l == F.n || hi - lo < 2 * FIX_FAN) {
        for (size_t i = lo; i < hi; i++) acc = xyzz_add(acc, at(i));
        break;
      }
      while (lo % FIX_FAN) acc = xyzz_add(acc, at(lo++));
      while (hi % FIX_FAN) acc = xyzz_add(acc, at(--hi));
      lo /= FIX_FAN;
      hi /= FIX_FAN;
      l++;
    }
    buckets[bk] = acc;
  }
}

// per (window, group): sum_{j in group} (j+1) B_j
__global__ void __launch_bounds__(256) k_bucket_reduce(const G1Xyzz *__restrict__ buckets, int W,
                                                       int half_buckets, int red_l, G1Xyzz *__restrict__ out) {
  const int groups = half_buckets / red_l;
  for (size_t id = blockIdx.x * (size_t)blockDim.x + threadIdx.x; id < (size_t)W * groups;
       id += (size_t)gridDim.x * blockDim.x) {
    int w = (int)(id / groups), g = (int)(id % groups);
    const G1Xyzz *B = buckets + (size_t)w * half_buckets;
    int a = g * red_l;
    G1Xyzz run = G1Xyzz::inf(), acc = G1Xyzz::inf();
    for (int j = a + red_l - 1; j >= a; j--) {
      run = xyzz_add(run, B[j]);
      acc = xyzz_add(acc, run);
    }
    if (a) acc = xyzz_add(acc, xyzz_mul_small(run, (uint64_t)a));
    out[id] = acc;
  }
}

// out[t] = sum of in[t*chunk .. (t+1)*chunk): shrinks the per-window partial count in
// parallel before the one-block-per-window tree (windows stay contiguous: chunk | groups).
__global__ void __launch_bounds__(256) k_sum_chunks(const G1Xyzz *__restrict__ in, size_t n_out, int chunk,
                                                    G1Xyzz *__restrict__ out) {
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < n_out; t += (size_t)gridDim.x * blockDim.x) {
    G1Xyzz acc = in[t * chunk];
    for (int i = 1; i < chunk; i++) acc = xyzz_add(acc, in[t * chunk + i]);
    out[t] = acc;
  }
}

__global__ void __launch_bounds__(256) k_window_sum(const G1Xyzz *__restrict__ parts, int groups,
                                                    G1Xyzz *__restrict__ out) {
  __shared__ G1Xyzz lds[256];
  const int w = blockIdx.x;
  G1Xyzz acc = G1Xyzz::inf();
  for (int g = threadIdx.x; g < groups; g += blockDim.x) acc = xyzz_add(acc, parts[(size_t)w * groups + g]);
  lds[threadIdx.x] = acc;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) lds[threadIdx.x] = xyzz_add(lds[threadIdx.x], lds[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) out[w] = lds[0];
}

// Naive path for tiny inputs: one thread per point, double-and-add, then a tree.
__global__ void __launch_bounds__(64) k_msm_tiny(const G1Affine *__restrict__ pts,
                                                 const Fr *__restrict__ scalars, int n,
                                                 G1Xyzz *__restrict__ out) {
  __shared__ G1Xyzz lds[64];
  G1Xyzz acc = G1Xyzz::inf();
  for (int i = threadIdx.x; i < n; i += 64) {
    Fr k = from_mont(scalars[i]);
    G1Xyzz r = G1Xyzz::inf();
    for (int b = 253; b >= 0; b--) {
      r = xyzz_dbl(r);
      if ((k.v[b >> 5] >> (b & 31)) & 1) r = xyzz_madd(r, pts[i]);
    }
    acc = xyzz_add(acc, r);
  }
  lds[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 32; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) lds[threadIdx.x] = xyzz_add(lds[threadIdx.x], lds[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = lds[0];
}

G1Xyzz msm_dev(Ctx *ctx, const G1Affine *points, const Fr *scalars, size_t n) {
  if (n == 0) return G1Xyzz::inf();
  hipStream_t st = ctx->stream;
  if (n <= 64) {
    G1Xyzz *d = (G1Xyzz *)ctx->msm_ws[0].ensure(sizeof(G1Xyzz));
    k_msm_tiny<<<1, 64, 0, st>>>(points, scalars, (int)n, d);
    TNS_LAUNCH_CHECK();
    G1Xyzz h;
    TNS_HIP(hipMemcpyAsync(&h, d, sizeof h, hipMemcpyDeviceToHost, st));
    TNS_HIP(hipStreamSynchronize(st));
    return h;
  }
  if (n >= ((size_t)1 << 31)) throw Error(TNS_ERR_COMMITMENT, "MSM larger than 2^31 points");
  unsigned bits = 0;
  {
    unsigned *d_bits = (unsigned *)ctx->msm_ws[4].ensure(sizeof(unsigned));
    TNS_HIP(hipMemsetAsync(d_bits, 0, sizeof(unsigned), st));
    k_scalar_bits<<<grid_for(n, 256, 2048), 256, 0, st>>>(scalars, n, d_bits);
    TNS_LAUNCH_CHECK();
    TNS_HIP(hipMemcpyAsync(&bits, d_bits, sizeof bits, hipMemcpyDeviceToHost, st));
    TNS_HIP(hipStreamSynchronize(st));
  }
  if (bits == 0) return G1Xyzz::inf();  // all scalars zero
  const MsmPlan P = make_plan(n, (int)bits);
  const size_t total = (size_t)P.W * n;
  if (total >= ((size_t)1 << 31)) throw Error(TNS_ERR_COMMITMENT, "MSM too large for one sort");
  const int half = 1 << (P.c - 1);

  uint32_t *keys = (uint32_t *)ctx->msm_ws[0].ensure(sizeof(uint32_t) * total);
  uint32_t *vals = (uint32_t *)ctx->msm_ws[1].ensure(sizeof(uint32_t) * total);
  uint32_t *keys2 = (uint32_t *)ctx->msm_ws[2].ensure(sizeof(uint32_t) * total);
  uint32_t *vals2 = (uint32_t *)ctx->msm_ws[3].ensure(sizeof(uint32_t) * total);
  uint32_t *bounds = (uint32_t *)ctx->msm_ws[4].ensure(sizeof(uint32_t) * (2 * P.nb + 1));
  uint32_t *bstart = bounds, *bend = bounds + P.nb, *valid = bounds + 2 * P.nb;
  G1Xyzz *buckets = (G1Xyzz *)ctx->msm_ws[5].ensure(sizeof(G1Xyzz) * P.nb);
  const size_t nchunks = (total + ACC_K - 1) / ACC_K;
  HeadTail *ht = (HeadTail *)ctx->msm_ws[6].ensure(sizeof(HeadTail) * nchunks);
  const int red_l = half < RED_L ? half : RED_L;
  const int groups = half / red_l;
  G1Xyzz *parts = (G1Xyzz *)ctx->msm_ws[7].ensure(sizeof(G1Xyzz) * (size_t)P.W * groups);
  G1Xyzz *wsum = (G1Xyzz *)ctx->msm_ws[8].ensure(sizeof(G1Xyzz) * P.W);

  {
    TNS_PROF(ctx, "msm_digits", 32.0 * n + 8.0 * total);
    k_digits<<<grid_for(n, 256), 256, 0, st>>>(scalars, n, P.c, P.W, P.sentinel, keys, vals);
    TNS_LAUNCH_CHECK();
  }

  size_t temp_bytes = 0;
  TNS_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, keys, keys2, vals, vals2, (int)total,
                                             0, P.end_bit, st));
  void *temp = ctx->msm_ws[9].ensure(temp_bytes);
  {
    TNS_PROF(ctx, "msm_sort", 16.0 * total);
    TNS_HIP(hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys, keys2, vals, vals2, (int)total, 0,
                                               P.end_bit, st));
  }

  TNS_HIP(hipMemsetAsync(bounds, 0, sizeof(uint32_t) * (2 * P.nb + 1), st));
  k_bucket_bounds<<<grid_for(total, 256), 256, 0, st>>>(keys2, total, P.sentinel, bstart, bend, valid);
  TNS_LAUNCH_CHECK();
  {
    TNS_PROF(ctx, "msm_accumulate", 96.0 * n);  // 96 B per (scalar, point) pair
    k_accumulate<<<grid_for(nchunks, 256, 1u << 30), 256, 0, st>>>(keys2, vals2, valid, bstart, bend,
                                                                   points, buckets, ht, nchunks);
    TNS_LAUNCH_CHECK();
  }
  {
    FixLevels F{};
    size_t groups = nchunks / FIX_FAN;
    size_t off = 0;
    while (F.n < FIX_LEVELS && groups >= 2) {  // level sizes: nchunks/32, /1024, ...
      F.len[F.n + 1] = groups;
      off += groups;
      groups /= FIX_FAN;
      F.n++;
    }
    TNS_PROF(ctx, "msm_fixup", 0.0);
    if (F.n) {
      G1Xyzz *base = (G1Xyzz *)ctx->fix_ws.ensure(sizeof(G1Xyzz) * off);
      size_t o = 0;
      for (int l = 1; l <= F.n; l++) {
        F.lv[l] = base + o;
        o += F.len[l];
        k_fix_level<<<grid_for(F.len[l], 256, 1u << 30), 256, 0, st>>>(keys2, valid, ht, F.lv[l - 1], l, F.len[l],
                                                                        F.lv[l]);
        TNS_LAUNCH_CHECK();
      }
    }
    k_bucket_fixup<<<grid_for(P.nb, 256), 256, 0, st>>>(bstart, bend, ht, F, buckets, P.nb);
    TNS_LAUNCH_CHECK();
  }
  {
    TNS_PROF(ctx, "msm_reduce", 128.0 * P.nb);
    k_bucket_reduce<<<grid_for((size_t)P.W * groups, 64, 1u << 30), 64, 0, st>>>(buckets, P.W, half, red_l,
                                                                                  parts);
    TNS_LAUNCH_CHECK();
    // shrink groups per window 16x per pass (ping-pong in the bucket array) down to <= 256
    G1Xyzz *src = parts, *dst = buckets;
    int g = groups;
    while (g > 256) {
      const int chunk = 16;
      const size_t n_out = (size_t)P.W * (g / chunk);
      k_sum_chunks<<<grid_for(n_out, 64, 1u << 30), 64, 0, st>>>(src, n_out, chunk, dst);
      TNS_LAUNCH_CHECK();
      std::swap(src, dst);
      g /= chunk;
    }
    k_window_sum<<<P.W, 256, 0, st>>>(src, g, wsum);
    TNS_LAUNCH_CHECK();
  }
  std::vector<G1Xyzz> S(P.W);
  TNS_HIP(hipMemcpyAsync(S.data(), wsum, sizeof(G1Xyzz) * P.W, hipMemcpyDeviceToHost, st));
  TNS_HIP(hipStreamSynchronize(st));
  G1Xyzz acc = S[P.W - 1];
  for (int w = P.W - 2; w >= 0; w--) {
    for (int k = 0; k < P.c; k++) acc = xyzz_dbl(acc);
    acc = xyzz_add(acc, S[w]);
  }
  return acc;
}

}  // namespace tns
