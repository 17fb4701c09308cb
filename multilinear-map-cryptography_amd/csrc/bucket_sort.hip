// bucket_sort.hip -- the MSM's (bucket, point) ordering: signed-window digits fused into a
// most-significant-digit-first counting sort.
//
// k_accumulate (msm.hip) needs the W*n (bucket, point|sign) entries of an MSM grouped by
// bucket.  A general radix sort (rocPRIM onesweep) spends a digit kernel, a histogram pass
// and one full read+write of keys and values per 8-bit digit on it.  Here:
//  * pass 1 reads the SCALARS (canonical, or Montgomery forms canonicalised on the fly, or raw
//    u64 trace values; 32 or 8 B for W entries), recomputes their digits in registers and scatters the entries straight into bins of the top key bits -- the
//    digit array never exists, and zero digits never enter the sort;
//  * passes 2.. split each bin by the next key bits.  MSD order needs no stability, so a
//    pass is per-tile LDS histograms + one exclusive scan + a scatter; tiles never cross a
//    bin, so a skewed bin (every scalar with the same digit) is just many tiles of one bin;
//  * every scatter first orders its tile by bin in LDS, then writes each bin's run with
//    consecutive lanes (coalesced stores instead of one scattered 4-B store per entry);
//  * the last pass's bin boundaries are the bucket bounds.
// Shared-bucket layout (fixed-base window tables): the key is (bucket, window), so inside a
// bucket the entries come window by window.  The accumulation gathers its points from the
// window's slab of the 12.9 GB table (T[w n + i]); window-major runs keep the slabs a wave
// touches at once few (entries of all 12 slabs mixed cost k_accumulate ~30 %).  The order
// inside one (bucket, window) run is unspecified (LDS atomics): bucket sums are group
// elements, so the MSM result does not depend on it.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "common.hpp"

namespace tns {

#ifndef TNS_BS_BLOCK
#define TNS_BS_BLOCK 256
#endif
constexpr int BS_BLOCK = TNS_BS_BLOCK;  // 4 waves: fits the slots k_accumulate leaves free
constexpr int BS_MAXBITS = 9;  // key bits per pass
constexpr int BS_MAXBINS = 1 << BS_MAXBITS;
#ifndef TNS_BS_TILE_MAX
#define TNS_BS_TILE_MAX 8192
#endif
constexpr int BS_TILE = TNS_BS_TILE_MAX;  // entries per tile at most (LDS staging: 8 B each, 64 KiB at 8192)
// per-pass tile sizes (template parameter TILE of the scatter kernels): 8192 or 4096 entries
constexpr int BS_SCALARS = 4;  // scalars a pass-1 thread loads ahead


struct DigitArgs {
  const Fr *scalars;
  size_t n, spb;  // scalars, scalars per tile (spb * W <= TILE)
  int c, W, wb;   // window bits, windows, window-index bits appended to the key (shared)
  bool shared;
  uint32_t stride;
  bool mont;             // scalars are Montgomery forms: canonicalised here
  const uint64_t *u64;   // set: raw u64 scalars instead (entries [0, n_u64), zero above)
  size_t n_u64;
};

// scalar i of the digit pass, canonical
__device__ __forceinline__ Fr load_scalar(const DigitArgs &A, size_t i) {
  if (A.u64) {
    const uint64_t x = i < A.n_u64 ? A.u64[i] : 0;
    Fr k = Fr::zero();
    k.v[0] = (uint32_t)x;
    k.v[1] = (uint32_t)(x >> 32);
    return k;
  }
  const Fr s = A.scalars[i];
  return A.mont ? from_mont(s) : s;
}

// signed c-bit digits of scalar i (msm.hip k_digits): f(key, value) for every non-zero digit;
// shared: key = (|d| - 1) << wb | w, value = (w * stride + i) | sign << 31
// per-window: key = w << (c - 1) | (|d| - 1), value = i | sign << 31
template <class F>
__device__ __forceinline__ void scalar_digits(const Fr &s, size_t i, const DigitArgs &A, F f) {
  const Fr &k = s;  // canonical (load_scalar)
  uint32_t carry = 0;
  const int c = A.c;
  const uint32_t half = 1u << (c - 1);
  for (int w = 0; w < A.W; w++) {
    const int bit = w * c;
    const int limb = bit >> 5, sh = bit & 31;
    uint64_t lo = 0, hi = 0;  // k.v[limb], k.v[limb + 1] by selects: a dynamic index would put
#pragma unroll                // the scalars in scratch memory
    for (int l = 0; l < 8; l++) {
      lo = l == limb ? k.v[l] : lo;
      hi = l == limb + 1 ? k.v[l] : hi;
    }
    const uint32_t raw = (uint32_t)(((lo | (hi << 32)) >> sh) & ((1u << c) - 1));
    const uint32_t val = raw + carry;
    uint32_t neg = 0, mag;
    if (val > half) {
      mag = (1u << c) - val;
      neg = 1;
      carry = 1;
    } else {
      mag = val;
      carry = 0;
    }
    if (mag) {
      const uint32_t key = A.shared ? ((mag - 1) << A.wb) | (uint32_t)w : ((uint32_t)w << (c - 1)) | (mag - 1);
      f(key, (uint32_t)(A.shared ? (size_t)w * A.stride + i : i) | (neg << 31));
    }
  }
}

// each thread's scalars of a pass-1 tile, BS_SCALARS loads in flight at a time
template <class F>
__device__ __forceinline__ void tile_scalars(const DigitArgs &A, size_t a, size_t b, F f) {
  for (size_t i0 = a + threadIdx.x; i0 < b; i0 += (size_t)BS_SCALARS * BS_BLOCK) {
    Fr s[BS_SCALARS];
#pragma unroll
    for (int j = 0; j < BS_SCALARS; j++) {
      const size_t i = i0 + (size_t)j * BS_BLOCK;
      if (i < b) s[j] = load_scalar(A, i);
    }
#pragma unroll
    for (int j = 0; j < BS_SCALARS; j++) {
      const size_t i = i0 + (size_t)j * BS_BLOCK;
      if (i < b) scalar_digits(s[j], i, A, f);
    }
  }
}

// The tile a scatter block works on.  Blocks are dealt round-robin over the 8 XCDs (blocks b and
// b + 8 share one, MI355X_MICROARCH.md), and consecutive tiles write adjacent runs into every bin
// (a run's last line is the next tile's first): TNS_BS_XCD builds map contiguous tile ranges to
// one XCD (the guide's bijective remap) so those shared lines merge in one L2 before write-back.
#ifndef TNS_BS_XCD
#define TNS_BS_XCD 0
#endif
__device__ __forceinline__ size_t scatter_tile() {
#if TNS_BS_XCD
  const size_t nwg = gridDim.x, orig = blockIdx.x, xcd = orig % 8, q = nwg / 8, r = nwg % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
#else
  return blockIdx.x;
#endif
}

// out[d] = sum_{d' < d} h[d'] for d < nb <= BPT * BS_BLOCK (BPT bins per thread)
template <int BPT = 2>
__device__ __forceinline__ void block_scan_bins(const uint32_t *h, uint32_t *out, int nb, uint32_t *wsum) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  uint32_t hv[BPT], mine = 0;
#pragma unroll
  for (int q = 0; q < BPT; q++) {
    hv[q] = BPT * t + q < nb ? h[BPT * t + q] : 0u;
    mine += hv[q];
  }
  uint32_t x = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  uint32_t off = 0;
  for (int i = 0; i < wv; i++) off += wsum[i];
  uint32_t ex = off + x - mine;
#pragma unroll
  for (int q = 0; q < BPT; q++) {
    if (BPT * t + q < nb) out[BPT * t + q] = ex;
    ex += hv[q];
  }
  __syncthreads();
}

static_assert(BS_MAXBINS <= 2 * BS_BLOCK, "two bins per thread in the block scan");

// Key formats between passes (BucketSortJob::kf): the keys a pass writes only need the key bits
// the later passes still sort by.  KF_U32: 4-byte keys; KF_U16: 2-byte keys (<= 16 bits left: the
// keys into the last pass, whose <= 9 key bits are all it reads).  (2-byte keys out of pass 1 too,
// the 17th bit carried in the value, measured slower: pass 1 +0.2 ms, pass 2 +0.35 ms per 2^24
// opening, their ~64-byte runs of half-dword stores costing more than the bytes saved.)
enum { KF_U32 = 0, KF_U16 = 1 };

// the scatters' stores (plain: non-temporal stores measured +1.3-2.1 ms per C4 step,
// profiles/r06_ab_sort_nt.txt)
template <class T>
__device__ __forceinline__ void st_out(T *p, T v) {
  *p = v;
}

__device__ __forceinline__ void store_entry(int kf, uint32_t *__restrict__ okeys, uint32_t *__restrict__ ovals,
                                            uint32_t pos, uint32_t key, uint32_t val) {
  if (kf == KF_U32) st_out(okeys + pos, key);
  else st_out(reinterpret_cast<uint16_t *>(okeys) + pos, (uint16_t)key);
  st_out(ovals + pos, val);
}

// entry i's key (the low bits a pass still needs) and value in format kf
__device__ __forceinline__ void load_entry(int kf, const uint32_t *__restrict__ keys, const uint32_t *__restrict__ vals,
                                           size_t i, uint32_t &key, uint32_t &val) {
  val = vals[i];
  key = kf == KF_U32 ? keys[i] : (uint32_t)reinterpret_cast<const uint16_t *>(keys)[i];
}

// key only (histograms)
__device__ __forceinline__ uint32_t load_key(int kf, const uint32_t *__restrict__ keys, size_t i) {
  return kf == KF_U32 ? keys[i] : (uint32_t)reinterpret_cast<const uint16_t *>(keys)[i];
}

// Tile writer: entries already placed in lk/lv by bin (bin d at [lbase[d], lbase[d] + cnt));
// consecutive lanes store consecutive slots of a bin's run at goff[d] + (slot - lbase[d]).
template <class BinOf>
__device__ __forceinline__ void write_tile(const uint32_t *lk, const uint32_t *lv, int m, const uint32_t *lbase,
                                           const uint32_t *goff, BinOf bin, int kf, uint32_t *__restrict__ okeys,
                                           uint32_t *__restrict__ ovals) {
  for (int slot = threadIdx.x; slot < m; slot += BS_BLOCK) {
    const uint32_t key = lk[slot];
    const uint32_t d = bin(key);
    const uint32_t pos = goff[d] + (uint32_t)slot - lbase[d];
    store_entry(kf, okeys, ovals, pos, key, lv[slot]);
  }
}

// pass 1 histogram: counts[d * T1 + tile] = entries of the tile with top digit d
__global__ void __launch_bounds__(BS_BLOCK) k_bs_count1(DigitArgs A, int shift, int nbins, size_t T1,
                                                        uint32_t *__restrict__ counts) {
  __shared__ uint32_t h[BS_MAXBINS];
  for (int d = threadIdx.x; d < nbins; d += BS_BLOCK) h[d] = 0;
  __syncthreads();
  const size_t tile = blockIdx.x, a = tile * A.spb, b = min(A.n, a + A.spb);
  tile_scalars(A, a, b, [&](uint32_t key, uint32_t) { atomicAdd(&h[key >> shift], 1u); });
  __syncthreads();
  for (int d = threadIdx.x; d < nbins; d += BS_BLOCK) counts[(size_t)d * T1 + tile] = h[d];
  if (tile == 0 && threadIdx.x == 0) counts[(size_t)nbins * T1] = 0;  // scan slot for the total
}

// pass 1 scatter: digits -> LDS ordered by bin -> coalesced runs
template <int TILE>
__global__ void __launch_bounds__(BS_BLOCK) k_bs_scatter1(DigitArgs A, int shift, int nbins, size_t T1,
                                                          const uint32_t *__restrict__ offs, int kf,
                                                          uint32_t *__restrict__ keys, uint32_t *__restrict__ vals) {
  __shared__ uint32_t h[BS_MAXBINS], lbase[BS_MAXBINS], goff[BS_MAXBINS], wsum[BS_BLOCK / 64];
  __shared__ uint32_t lk[TILE], lv[TILE];
  const size_t tile = scatter_tile(), a = tile * A.spb, b = min(A.n, a + A.spb);
  for (int d = threadIdx.x; d < nbins; d += BS_BLOCK) {
    h[d] = 0;
    goff[d] = offs[(size_t)d * T1 + tile];
  }
  __syncthreads();
  tile_scalars(A, a, b, [&](uint32_t key, uint32_t) { atomicAdd(&h[key >> shift], 1u); });
  __syncthreads();
  block_scan_bins(h, lbase, nbins, wsum);
  for (int d = threadIdx.x; d < nbins; d += BS_BLOCK) h[d] = lbase[d];  // cursors
  __syncthreads();
  tile_scalars(A, a, b, [&](uint32_t key, uint32_t val) {  // second digit sweep (scalars are cached)
    const uint32_t slot = atomicAdd(&h[key >> shift], 1u);
    lk[slot] = key;
    lv[slot] = val;
  });
  __syncthreads();
  const int m = (int)h[nbins - 1];  // the last bin's cursor ends at the tile's entry count
  write_tile(lk, lv, m, lbase, goff, [&](uint32_t key) { return key >> shift; }, kf, keys, vals);
}

// ---- pass 1 with a compile-time window plan (C bits, W windows): the digit of window w sits
// at a constant bit offset, so it is one funnel shift of two known limbs (the runtime plan
// needs 16 selects per window to avoid a dynamic register index), and each thread keeps its
// entries' keys and LDS ranks in registers: ONE digit sweep and ONE returning LDS atomic per
// entry (the runtime kernels sweep twice and count twice).  Each thread owns up to SPT
// scalars of the tile (tile = spb <= 256 SPT scalars, spb W <= TILE entries).
template <int C, int W>
__device__ __forceinline__ uint32_t digit_raw(const Fr &k, int w) {
  const int bit = w * C, limb = bit >> 5, sh = bit & 31;
  const uint32_t lo = limb < 8 ? k.v[limb] : 0u, hi = limb + 1 < 8 ? k.v[limb + 1] : 0u;
  const uint32_t x = sh ? (uint32_t)((((uint64_t)hi << 32) | lo) >> sh) : lo;
  return x & ((1u << C) - 1);
}

// signed digits of one scalar: g(w, key, neg) for every non-zero digit (keys as scalar_digits)
template <int C, int W, class G>
__device__ __forceinline__ void scalar_digits_ct(const Fr &k, const DigitArgs &A, G g) {
  constexpr uint32_t half = 1u << (C - 1);
  uint32_t carry = 0;
#pragma unroll
  for (int w = 0; w < W; w++) {
    const uint32_t val = digit_raw<C, W>(k, w) + carry;
    const bool negd = val > half;
    const uint32_t mag = negd ? (1u << C) - val : val;
    carry = negd ? 1u : 0u;
    if (mag) {
      const uint32_t key = A.shared ? ((mag - 1) << A.wb) | (uint32_t)w : ((uint32_t)w << (C - 1)) | (mag - 1);
      g(w, key, negd);
    }
  }
}

// bits (optional): also the largest bit length of the (canonical) scalars -- the MSM's plan input,
// computed here when the plan was known ahead (bucket_sort_precount_bits) instead of by k_scalar_bits
// low64 (optional, with bits): each scalar's canonical low 64 bits (the sort's narrow input, below)
template <int C, int W>
__global__ void __launch_bounds__(BS_BLOCK) k_bs_count1_ct(DigitArgs A, int shift, int nbins, size_t T1,
                                                           uint32_t *__restrict__ counts, unsigned *bits,
                                                           uint64_t *__restrict__ low64) {
  __shared__ uint32_t h[BS_MAXBINS];
  for (int d = threadIdx.x; d < nbins; d += BS_BLOCK) h[d] = 0;
  __syncthreads();
  const size_t tile = blockIdx.x, a = tile * A.spb, b = min(A.n, a + A.spb);
  unsigned bl = 0;
  for (size_t i0 = a + threadIdx.x; i0 < b; i0 += (size_t)BS_SCALARS * BS_BLOCK) {
    Fr s[BS_SCALARS];  // the loads in flight together, then the digits
#pragma unroll
    for (int j = 0; j < BS_SCALARS; j++)
      if (i0 + (size_t)j * BS_BLOCK < b) s[j] = load_scalar(A, i0 + (size_t)j * BS_BLOCK);
#pragma unroll
    for (int j = 0; j < BS_SCALARS; j++)
      if (i0 + (size_t)j * BS_BLOCK < b) {
        if (bits) bl = max(bl, fr_bit_length(s[j]));
        if (low64) low64[i0 + (size_t)j * BS_BLOCK] = (uint64_t)s[j].v[0] | ((uint64_t)s[j].v[1] << 32);
        scalar_digits_ct<C, W>(s[j], A, [&](int, uint32_t key, bool) { atomicAdd(&h[key >> shift], 1u); });
      }
  }
  __syncthreads();
  for (int d = threadIdx.x; d < nbins; d += BS_BLOCK) counts[(size_t)d * T1 + tile] = h[d];
  if (tile == 0 && threadIdx.x == 0) counts[(size_t)nbins * T1] = 0;
  if (bits) block_atomic_max2(bl, 0u, bits, nullptr);
}

constexpr uint32_t BS_NOKEY = 0x40000000u;  // empty entry slot (keys are < 2^30; bit 31 = sign)

template <int TILE, int C, int W, int SPT>
__global__ void __launch_bounds__(BS_BLOCK) k_bs_scatter1_ct(DigitArgs A, int shift, int nbins, size_t T1,
                                                             const uint32_t *__restrict__ offs, int kf,
                                                             uint32_t *__restrict__ keys, uint32_t *__restrict__ vals) {
  __shared__ uint32_t h[BS_MAXBINS], lbase[BS_MAXBINS], goff[BS_MAXBINS], wsum[BS_BLOCK / 64];
  __shared__ uint32_t lk[TILE], lv[TILE];
  const size_t tile = scatter_tile(), a = tile * A.spb, b = min(A.n, a + A.spb);
  for (int d = threadIdx.x; d < nbins; d += BS_BLOCK) {
    h[d] = 0;
    goff[d] = offs[(size_t)d * T1 + tile];
  }
  __syncthreads();
  uint32_t ek[SPT][W], er[SPT][W];  // key | sign << 31 (BS_NOKEY: none), rank inside its bin
  constexpr int LA = SPT < BS_SCALARS ? SPT : BS_SCALARS;  // scalar loads in flight together
  Fr s[LA];
#pragma unroll
  for (int j = 0; j < SPT; j++) {
    if (j % LA == 0) {
#pragma unroll
      for (int q = 0; q < LA; q++) {
        const size_t iq = a + threadIdx.x + (size_t)(j + q) * BS_BLOCK;
        if (j + q < SPT && iq < b) s[q] = load_scalar(A, iq);
      }
    }
#pragma unroll
    for (int w = 0; w < W; w++) ek[j][w] = BS_NOKEY;
    const size_t i = a + threadIdx.x + (size_t)j * BS_BLOCK;
    if (i < b)
      scalar_digits_ct<C, W>(s[j % LA], A, [&](int w, uint32_t key, bool negd) {
        er[j][w] = atomicAdd(&h[key >> shift], 1u);
        ek[j][w] = key | (negd ? 0x80000000u : 0u);
      });
  }
  __syncthreads();
  block_scan_bins(h, lbase, nbins, wsum);
  const int m = (int)(lbase[nbins - 1] + h[nbins - 1]);
#pragma unroll
  for (int j = 0; j < SPT; j++) {
    const size_t i = a + threadIdx.x + (size_t)j * BS_BLOCK;
#pragma unroll
    for (int w = 0; w < W; w++) {
      const uint32_t e = ek[j][w];
      if (e != BS_NOKEY) {
        const uint32_t key = e & 0x7fffffffu;
        const uint32_t slot = lbase[key >> shift] + er[j][w];
        lk[slot] = key;
        lv[slot] = (uint32_t)(A.shared ? (size_t)w * A.stride + i : i) | (e & 0x80000000u);
      }
    }
  }
  __syncthreads();
  write_tile(lk, lv, m, lbase, goff, [&](uint32_t key) { return key >> shift; }, kf, keys, vals);
}

// compile-time plans of the pass-1 kernels: the fixed-base table windows (n = 2^20..2^26) and
// the narrow trace commitments' per-window plans; anything else takes the runtime kernels
struct Pass1Plan {
  int tile, c, W;
  void (*count)(DigitArgs, int, int, size_t, uint32_t *, unsigned *, uint64_t *);
  void (*scatter)(DigitArgs, int, int, size_t, const uint32_t *, int, uint32_t *, uint32_t *);
  int spt;
};
#define TNS_P1(T, C, W, SPT) {T, C, W, k_bs_count1_ct<C, W>, k_bs_scatter1_ct<T, C, W, SPT>, SPT}
static const Pass1Plan kPass1Plans[] = {
    TNS_P1(BS_TILE, 22, 12, 3), TNS_P1(BS_TILE, 20, 13, 3), TNS_P1(BS_TILE, 19, 14, 3),
    TNS_P1(BS_TILE, 17, 15, 3), TNS_P1(BS_TILE, 16, 2, 16), TNS_P1(BS_TILE, 12, 2, 16)};
#undef TNS_P1

// bins of pass 1 -> segment starts; seg[nbins] = total = number of entries (also *valid)
__global__ void k_bs_segs1(const uint32_t *__restrict__ offs, int nbins, size_t T1, uint32_t *__restrict__ seg,
                           uint32_t *__restrict__ valid) {
  for (int d = threadIdx.x; d <= nbins; d += blockDim.x) seg[d] = offs[(size_t)d * T1];
  if (threadIdx.x == 0) {
    valid[0] = offs[(size_t)nbins * T1];
    valid[1] = 0;  // (k_accumulate sets it when a run crosses a chunk)
  }
}

// tiles per segment
// tiles per segment; mcount (optional): the same for segments of >= 2 tiles, else 0
__global__ void k_bs_tiles(const uint32_t *__restrict__ seg, size_t S, uint32_t tile, uint32_t *__restrict__ tcount,
                           uint32_t *__restrict__ mcount) {
  for (size_t s = blockIdx.x * (size_t)blockDim.x + threadIdx.x; s <= S; s += (size_t)gridDim.x * blockDim.x) {
    const uint32_t t = s < S ? (uint32_t)((seg[s + 1] - seg[s] + tile - 1) / tile) : 0u;
    tcount[s] = t;
    if (mcount) mcount[s] = t > 1 ? t : 0u;
  }
}

// desc[tile_base[s] + k] = s for the tiles k of segment s: one thread per tile, a binary search of
// the tile bases (a thread per segment walked up to ~3 K tiles of one segment: 0.18 ms at 2^24)
__global__ void k_bs_desc(const uint32_t *__restrict__ tbase, size_t S, uint32_t *__restrict__ desc) {
  const uint32_t ntiles = tbase[S];
  for (size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x; g < ntiles; g += (size_t)gridDim.x * blockDim.x) {
    size_t lo = 0, hi = S;  // the last s with tbase[s] <= g (empty segments repeat the next base)
    while (hi - lo > 1) {
      const size_t mid = (lo + hi) >> 1;
      if (tbase[mid] <= g) lo = mid;
      else hi = mid;
    }
    desc[g] = (uint32_t)lo;
  }
}

struct PassGeom {
  const uint32_t *seg, *tbase, *desc;
  int shift, nbins;
  uint32_t mask;
  int ident;              // every segment is one tile: tile g = segment g (tbase / desc unused)
  const uint32_t *mbase;  // set: the counts hold only segments of >= 2 tiles, segment s's block at
                          // nbins * mbase[s] (exclusive scan of their tile counts); else at nbins * tbase[s]
  int kin, kout;          // key formats read and written (KF_*)
};

// the first count slot of segment s (its first tile tb)
__device__ __forceinline__ size_t count_base(const PassGeom &G, uint32_t s, uint32_t tb) {
  return (size_t)G.nbins * (G.mbase ? G.mbase[s] : tb);
}

// tile g's segment s, the segment's first tile tb and its tile count Ts
__device__ __forceinline__ void tile_geom(const PassGeom &G, size_t g, uint32_t &s, uint32_t &tb, uint32_t &Ts) {
  if (G.ident) {
    s = tb = (uint32_t)g;
    Ts = 1;
  } else {
    s = G.desc[g];
    tb = G.tbase[s];
    Ts = G.tbase[s + 1] - tb;
  }
}


// passes >= 2, histogram: counts[nbins * tbase[s] + d * T_s + k]
template <int TILE, int NB = BS_MAXBINS>
__global__ void __launch_bounds__(BS_BLOCK) k_bs_count(PassGeom G, size_t S, size_t max_tiles,
                                                       const uint32_t *__restrict__ keys, uint32_t *__restrict__ counts) {
  __shared__ uint32_t h[NB];
  const size_t g = blockIdx.x;
  if (!G.mbase) {  // full layout over max_tiles slots (the compact one is sized exactly by the host)
    if (g == max_tiles - 1 && threadIdx.x == 0) counts[(size_t)G.nbins * max_tiles] = 0;
    if (g >= G.tbase[S]) {  // unused tile slot: zero its share of the scan input
      for (int d = threadIdx.x; d < G.nbins; d += BS_BLOCK) counts[(size_t)G.nbins * g + d] = 0;
      return;
    }
  }
  for (int d = threadIdx.x; d < G.nbins; d += BS_BLOCK) h[d] = 0;
  __syncthreads();
  uint32_t s, tb, Ts;
  tile_geom(G, g, s, tb, Ts);
  const uint32_t k = (uint32_t)g - tb;
  if (Ts == 1) {  // a one-tile segment: k_bs_scatter ranks it locally (no keys read here)
    if (!G.mbase)
      for (int d = threadIdx.x; d < G.nbins; d += BS_BLOCK) counts[(size_t)G.nbins * tb + d] = 0;
    return;
  }
  constexpr int IPT = TILE / BS_BLOCK;
  const size_t a = G.seg[s] + (size_t)k * TILE, e = min((size_t)G.seg[s + 1], a + TILE);
  uint32_t kk[IPT];
  // the format branch outside the loads: one branch per load would serialise them
  auto loads = [&](auto kin) {
#pragma unroll
    for (int j = 0; j < IPT; j++) {
      const size_t p = a + threadIdx.x + (size_t)j * BS_BLOCK;
      kk[j] = p < e ? load_key(decltype(kin)::value, keys, p) : 0;
    }
  };
  if (G.kin == KF_U32) loads(std::integral_constant<int, KF_U32>());
  else loads(std::integral_constant<int, KF_U16>());
#pragma unroll
  for (int j = 0; j < IPT; j++)
    if (a + threadIdx.x + (size_t)j * BS_BLOCK < e) atomicAdd(&h[(kk[j] >> G.shift) & G.mask], 1u);
  __syncthreads();
  const size_t cb = count_base(G, s, tb);
  for (int d = threadIdx.x; d < G.nbins; d += BS_BLOCK) counts[cb + (size_t)d * Ts + k] = h[d];
}

// Packed tail of the sort (BucketSortJob::pk): after the second-to-last pass an entry needs only
// the last pass's L key bits, its sign and its point index i (ibits bits), so that pass writes
// them as one word  x = key_low << (ibits + 1) | sign << ibits | i  (4 bytes instead of a key and
// a value), the last pass bins x by its top bits and writes the accumulation's value alone
// (w stride + i | sign << 31; w = the key's window bits): 4 bytes fewer per entry written by the
// second-to-last pass and read by the last.  Used when the usual split leaves room (n <= 2^22).
// Independently, the last pass of every multi-pass sort writes the values only (PK 3): the
// accumulation finds its runs from the bucket starts instead of a key per entry.
struct PackArgs {
  int ibits, L, wb, shared;
  uint32_t stride;
};

// PK 0: keys + values in and out; 1: keys + values in, packed words out (okeys);
// 2: packed words in (keys), values out (ovals); 3: keys + values in, values out
__device__ __forceinline__ uint32_t pack_entry(const PackArgs &P, uint32_t key, uint32_t v) {
  const uint32_t i = P.shared ? (v & 0x7fffffffu) - (key & ((1u << P.wb) - 1)) * P.stride : (v & 0x7fffffffu);
  return ((key & ((1u << P.L) - 1)) << (P.ibits + 1)) | ((v >> 31) << P.ibits) | i;
}
__device__ __forceinline__ uint32_t unpack_value(const PackArgs &P, uint32_t x) {
  const uint32_t i = x & ((1u << P.ibits) - 1), sign = (x >> P.ibits) & 1u;
  const uint32_t w = P.shared ? (x >> (P.ibits + 1)) & ((1u << P.wb) - 1) : 0u;
  return (w * P.stride + i) | (sign << 31);
}

// passes >= 2, scatter: tile -> LDS ordered by bin -> coalesced runs.  Segment s's block of
// the scanned counts starts at offs[nbins tb]; one-tile segments (the common case in the last
// pass) have zero counts there and take their bin offsets, and the next pass's segment
// starts, from their own LDS scan.
template <int TILE, int PK, int NB = BS_MAXBINS>
__global__ void __launch_bounds__(BS_BLOCK) k_bs_scatter(PassGeom G, size_t S, const uint32_t *__restrict__ offs,
                                                         const uint32_t *__restrict__ keys,
                                                         const uint32_t *__restrict__ vals,
                                                         uint32_t *__restrict__ okeys, uint32_t *__restrict__ ovals,
                                                         uint32_t *__restrict__ nseg, PackArgs P) {
  __shared__ uint32_t h[NB], lbase[NB], goff[NB], wsum[BS_BLOCK / 64];
  constexpr int IPT = TILE / BS_BLOCK;
  __shared__ uint32_t lk[TILE], lv[PK == 2 ? 1 : TILE];
  const size_t g = scatter_tile();
  if (g >= (G.ident ? S : G.tbase[S])) return;
  uint32_t s, tb, Ts;
  tile_geom(G, g, s, tb, Ts);
  const uint32_t k = (uint32_t)g - tb;
  const uint32_t s0 = G.seg[s];
  const size_t cb = Ts == 1 ? 0 : count_base(G, s, tb);
  const uint32_t base = Ts == 1 ? 0u : s0 - offs[cb];
  for (int d = threadIdx.x; d < G.nbins; d += BS_BLOCK) {
    h[d] = 0;
    if (Ts != 1) goff[d] = base + offs[cb + (size_t)d * Ts + k];
  }
  const size_t a = s0 + (size_t)k * TILE, e = min((size_t)G.seg[s + 1], a + TILE);
  const int m = (int)(e - a);
  uint32_t kk[IPT], vv[IPT], rk[IPT];
  auto loads = [&](auto kin) {  // (the format branch outside the loads, as in k_bs_count)
#pragma unroll
    for (int j = 0; j < IPT; j++) {
      const int q = threadIdx.x + j * BS_BLOCK;
      if (q < m) {
        if (PK == 2) kk[j] = keys[a + q];
        else load_entry(decltype(kin)::value, keys, vals, a + q, kk[j], vv[j]);
      }
    }
  };
  if (PK == 2 || G.kin == KF_U32) loads(std::integral_constant<int, KF_U32>());
  else loads(std::integral_constant<int, KF_U16>());
  __syncthreads();
#pragma unroll
  for (int j = 0; j < IPT; j++)
    if ((int)threadIdx.x + j * BS_BLOCK < m) rk[j] = atomicAdd(&h[(kk[j] >> G.shift) & G.mask], 1u);
  __syncthreads();
  block_scan_bins<NB / BS_BLOCK>(h, lbase, G.nbins, wsum);
  if (Ts == 1)
    for (int d = threadIdx.x; d < G.nbins; d += BS_BLOCK) {
      goff[d] = s0 + lbase[d];
      nseg[(size_t)s * G.nbins + d] = s0 + lbase[d];
    }
#pragma unroll
  for (int j = 0; j < IPT; j++) {
    if ((int)threadIdx.x + j * BS_BLOCK < m) {
      const uint32_t slot = lbase[(kk[j] >> G.shift) & G.mask] + rk[j];
      lk[slot] = kk[j];
      if (PK != 2) lv[slot] = vv[j];
    }
  }
  __syncthreads();
  for (int slot = threadIdx.x; slot < m; slot += BS_BLOCK) {  // coalesced runs (write_tile)
    const uint32_t key = lk[slot];
    const uint32_t d = (key >> G.shift) & G.mask;
    const uint32_t pos = goff[d] + (uint32_t)slot - lbase[d];
    if (PK == 0) {
      store_entry(G.kout, okeys, ovals, pos, key, lv[slot]);
    } else if (PK == 3) {
      st_out(ovals + pos, lv[slot]);
    } else if (PK == 1) {
      st_out(okeys + pos, pack_entry(P, key, lv[slot]));
    } else {
      st_out(ovals + pos, unpack_value(P, key));
    }
  }
}

// new segments s * nbins + d: their starts; nseg[S * nbins] = end of the last segment
// (one-tile segments: written by k_bs_scatter)
__global__ void k_bs_segs(PassGeom G, size_t S, const uint32_t *__restrict__ offs, uint32_t *__restrict__ nseg) {
  const size_t NS = S * (size_t)G.nbins;
  for (size_t id = blockIdx.x * (size_t)blockDim.x + threadIdx.x; id <= NS; id += (size_t)gridDim.x * blockDim.x) {
    if (id == NS) {
      nseg[NS] = G.seg[S];
      continue;
    }
    if (G.ident) continue;  // every segment was ranked locally (k_bs_scatter wrote nseg)
    const size_t s = id / G.nbins, d = id % G.nbins;
    const uint32_t tb = G.tbase[s], Ts = G.tbase[s + 1] - tb;
    if (Ts == 1) continue;
    const size_t cb = count_base(G, (uint32_t)s, tb);
    nseg[id] = Ts ? G.seg[s] + (offs[cb + d * Ts] - offs[cb]) : G.seg[s];
  }
}

// bucket bounds from the (bucket, window) segment starts: out[b] = seg[b << wb], b <= nb
__global__ void k_bs_bucket_starts(const uint32_t *__restrict__ seg, size_t nb, int wb, uint32_t *__restrict__ out) {
  for (size_t b = blockIdx.x * (size_t)blockDim.x + threadIdx.x; b <= nb; b += (size_t)gridDim.x * blockDim.x)
    out[b] = seg[b << wb];
}

// ---- exclusive scan of u32 counts (the sort's bin offsets): tiles of 4096 (256 threads x 16
// consecutive items), reduce -> one block scanning the tile sums -> apply; a single tile is one
// launch.  Replaces rocPRIM's look-back scan (round 3: 432 library launches per step).
constexpr int SCAN_THREADS = 256, SCAN_ITEMS = 16, SCAN_TILE = SCAN_THREADS * SCAN_ITEMS;
// The one-block kernels of the sort's geometry (k_scan_parts, k_scan_single, k_bs_geom) run while
// the OTHER lane's scatter holds most of every CU: a 1024-thread block needs 16 free wave slots on
// one CU and waited for that scatter to drain (0.44-0.52 ms per launch in the C4 timeline,
// profiles/r06_c4_step_timeline_p1.txt), 256-thread blocks slip in beside it.
constexpr int ONE_BLOCK = 256;

// exclusive prefix of x over the block (NT threads); *sum = the block total.  lds: NT / 64 words
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t *lds, uint32_t &sum) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) lds[w] = inc;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; i++) {
    const uint32_t v = lds[i];
    off += i < w ? v : 0u;
    tot += v;
  }
  __syncthreads();  // lds free for the caller's next scan
  sum = tot;
  return off + inc - x;
}

// thread's SCAN_ITEMS consecutive items of the tile (zeros past n)
__device__ __forceinline__ void scan_load(const uint32_t *__restrict__ in, size_t n, size_t base, uint32_t (&x)[SCAN_ITEMS]) {
  if (base + SCAN_ITEMS <= n && (reinterpret_cast<uintptr_t>(in) & 15) == 0) {
    const uint4 *p = reinterpret_cast<const uint4 *>(in + base);  // base is a multiple of 16 items
#pragma unroll
    for (int q = 0; q < SCAN_ITEMS / 4; q++) {
      const uint4 v = p[q];
      x[4 * q] = v.x;
      x[4 * q + 1] = v.y;
      x[4 * q + 2] = v.z;
      x[4 * q + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) x[k] = base + k < n ? in[base + k] : 0u;
  }
}

__global__ void __launch_bounds__(SCAN_THREADS) k_scan_reduce(const uint32_t *__restrict__ in, size_t n,
                                                              uint32_t *__restrict__ part) {
  __shared__ uint32_t lds[SCAN_THREADS / 64];
  uint32_t x[SCAN_ITEMS];
  scan_load(in, n, (size_t)blockIdx.x * SCAN_TILE + (size_t)threadIdx.x * SCAN_ITEMS, x);
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; k++) s += x[k];
  uint32_t tot;
  (void)block_excl_scan<SCAN_THREADS>(s, lds, tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// the tile sums, scanned in place by one block
__global__ void __launch_bounds__(ONE_BLOCK) k_scan_parts(uint32_t *__restrict__ part, size_t np) {
  __shared__ uint32_t lds[ONE_BLOCK / 64];
  uint32_t carry = 0;
  for (size_t b0 = 0; b0 < np; b0 += ONE_BLOCK) {
    const size_t i = b0 + threadIdx.x;
    const uint32_t x = i < np ? part[i] : 0u;
    uint32_t tot;
    const uint32_t pre = block_excl_scan<ONE_BLOCK>(x, lds, tot);
    if (i < np) part[i] = carry + pre;
    carry += tot;
  }
}

__global__ void __launch_bounds__(SCAN_THREADS) k_scan_apply(const uint32_t *__restrict__ in, size_t n,
                                                             const uint32_t *__restrict__ part,
                                                             uint32_t *__restrict__ out) {
  __shared__ uint32_t lds[SCAN_THREADS / 64];
  const size_t base = (size_t)blockIdx.x * SCAN_TILE + (size_t)threadIdx.x * SCAN_ITEMS;
  uint32_t x[SCAN_ITEMS];
  scan_load(in, n, base, x);
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; k++) {
    const uint32_t v = x[k];
    x[k] = s;  // in-thread exclusive prefix
    s += v;
  }
  uint32_t tot;
  const uint32_t off = (part ? part[blockIdx.x] : 0u) + block_excl_scan<SCAN_THREADS>(s, lds, tot);
  if (base + SCAN_ITEMS <= n && (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
    uint4 *o = reinterpret_cast<uint4 *>(out + base);
#pragma unroll
    for (int q = 0; q < SCAN_ITEMS / 4; q++)
      o[q] = make_uint4(off + x[4 * q], off + x[4 * q + 1], off + x[4 * q + 2], off + x[4 * q + 3]);
  } else {
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++)
      if (base + k < n) out[base + k] = off + x[k];
  }
}

// up to SCAN_SMALL counts in ONE launch: one block of ONE_BLOCK threads walks the array in rounds of
// ONE_BLOCK x 16 (the segment-count scans of the later passes, where three launches of a few
// microseconds each were most of the cost).  2^15: the last pass of a 2^24-scalar opening MSM has
// 65 537 segments, whose one-block geometry took ~0.3 ms beside the other lane's scatter (16 serial
// rounds); the multi-block tiles + scans take ~0.1 ms (C4 -0.17 ms, profiles/r06_ab_sort_geom_threshold.txt)
#ifndef TNS_SCAN_SMALL_LOG  // (build-time A/B only)
#define TNS_SCAN_SMALL_LOG 15
#endif
constexpr size_t SCAN_SMALL = (size_t)1 << TNS_SCAN_SMALL_LOG;
__global__ void __launch_bounds__(ONE_BLOCK) k_scan_single(const uint32_t *__restrict__ in, size_t n,
                                                      uint32_t *__restrict__ out) {
  __shared__ uint32_t lds[ONE_BLOCK / 64];
  uint32_t carry = 0;
  for (size_t b0 = 0; b0 < n; b0 += (size_t)ONE_BLOCK * SCAN_ITEMS) {
    const size_t base = b0 + (size_t)threadIdx.x * SCAN_ITEMS;
    uint32_t x[SCAN_ITEMS];
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) x[k] = base + k < n ? in[base + k] : 0u;
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) {
      const uint32_t v = x[k];
      x[k] = s;
      s += v;
    }
    uint32_t tot;
    const uint32_t off = carry + block_excl_scan<ONE_BLOCK>(s, lds, tot);
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++)
      if (base + k < n) out[base + k] = off + x[k];
    carry += tot;
  }
}

// A pass's tile geometry in ONE launch (segments S + 1 <= SCAN_SMALL): tbase = exclusive scan of
// the tiles per segment (and mbase: of the tiles of segments with >= 2 of them), computed straight
// from the segment starts -- k_bs_tiles + one or two scans were 3-4 launches of ~5-17 us.  pub
// (the last pass): the two totals and the entry count go to the lane's host buffer with a flag.
__global__ void __launch_bounds__(ONE_BLOCK) k_bs_geom(const uint32_t *__restrict__ seg, size_t S, uint32_t tile,
                                                  uint32_t *__restrict__ tbase, uint32_t *__restrict__ mbase,
                                                  const uint32_t *__restrict__ valid, uint32_t *pub, uint32_t *flag,
                                                  uint32_t seq) {
  __shared__ uint32_t lds[ONE_BLOCK / 64], lds2[ONE_BLOCK / 64];
  const size_t n = S + 1;
  uint32_t ct = 0, cm = 0;
  for (size_t b0 = 0; b0 < n; b0 += (size_t)ONE_BLOCK * SCAN_ITEMS) {
    const size_t base = b0 + (size_t)threadIdx.x * SCAN_ITEMS;
    uint32_t xt[SCAN_ITEMS], xm[SCAN_ITEMS], st = 0, sm = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) {
      const size_t i = base + k;
      const uint32_t t = i < S ? (seg[i + 1] - seg[i] + tile - 1) / tile : 0u;
      xt[k] = st;
      st += t;
      xm[k] = sm;
      sm += t > 1 ? t : 0u;
    }
    uint32_t tot_t, tot_m = 0;
    const uint32_t off_t = ct + block_excl_scan<ONE_BLOCK>(st, lds, tot_t);
    const uint32_t off_m = mbase ? cm + block_excl_scan<ONE_BLOCK>(sm, lds2, tot_m) : 0u;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++)
      if (base + k < n) {
        tbase[base + k] = off_t + xt[k];
        if (mbase) mbase[base + k] = off_m + xm[k];
      }
    ct += tot_t;
    cm += tot_m;
  }
  if (pub && threadIdx.x == 0) {
    pub[0] = ct;  // = tbase[S]
    pub[1] = cm;  // = mbase[S]
    pub[2] = *valid;
    __threadfence_system();
    __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// out[i] = sum_{j < i} in[j] for i < n (in and out distinct device arrays; 16-byte vector
// loads / stores where the array is 16-byte aligned)
static void exclusive_scan(hipStream_t st, DevBuf &tmp, const uint32_t *in, uint32_t *out, size_t n) {
  if (!n) return;
  const size_t tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
  if (tiles == 1) {
    k_scan_apply<<<1, SCAN_THREADS, 0, st>>>(in, n, nullptr, out);
    TNS_LAUNCH_CHECK();
    return;
  }
  if (n <= SCAN_SMALL) {
    k_scan_single<<<1, ONE_BLOCK, 0, st>>>(in, n, out);
    TNS_LAUNCH_CHECK();
    return;
  }
  uint32_t *part = (uint32_t *)tmp.ensure(sizeof(uint32_t) * tiles);
  k_scan_reduce<<<(unsigned)tiles, SCAN_THREADS, 0, st>>>(in, n, part);
  TNS_LAUNCH_CHECK();
  k_scan_parts<<<1, ONE_BLOCK, 0, st>>>(part, tiles);
  TNS_LAUNCH_CHECK();
  k_scan_apply<<<(unsigned)tiles, SCAN_THREADS, 0, st>>>(in, n, part, out);
  TNS_LAUNCH_CHECK();
}

// Pass 1's geometry for W*n entries of `bucket_bits`-bit buckets: key bits and passes, the
// compile-time plan (if any), scalars per tile, tiles, bins, shift and the count buffer's length
struct Pass1Geom {
  int keybits = 0, npass = 0, wb = 0, bits0 = 0, nb = 0, shift = 0;
  const Pass1Plan *ct = nullptr;
  size_t spb = 0, T1 = 0, cnt_len = 0;
};
static Pass1Geom pass1_geom(size_t n, int c, int W, bool shared, int bucket_bits) {
  Pass1Geom g;
  if (shared)
    while ((1 << g.wb) < W) g.wb++;
  g.keybits = bucket_bits + g.wb;
  g.npass = std::max(1, (g.keybits + BS_MAXBITS - 1) / BS_MAXBITS);
  // the last pass sorts LDS-sized segments by BS_MAXBITS bits; the passes before it split the
  // remaining bits evenly (25-bit keys: 8, 8, 9 -- pass 2 with 256 instead of 512 bins writes
  // 128-byte runs: 1.21 -> 1.02 ms at 2^24)
  const int last = std::min(g.keybits, BS_MAXBITS);
  g.bits0 = g.npass == 1 ? last : (g.keybits - last + (g.npass - 2)) / (g.npass - 1);
  g.nb = 1 << g.bits0;
  g.shift = g.keybits - g.bits0;
  for (const Pass1Plan &p : kPass1Plans)
    if (p.tile == BS_TILE && p.c == c && p.W == W) g.ct = &p;
  g.spb = (size_t)BS_TILE / W;
  if (g.ct) g.spb = std::min(g.spb, (size_t)BS_BLOCK * g.ct->spt);
  g.T1 = (n + g.spb - 1) / g.spb;
  const size_t E = (size_t)W * n, max_seg = (size_t)1 << g.keybits, tmin = 4096;
  const size_t max_tiles = (E + tmin - 1) / tmin + (max_seg >> last) + 1;
  g.cnt_len = std::max((size_t)g.nb * g.T1, (size_t)BS_MAXBINS * max_tiles) + 1;
  return g;
}

// Groups the W*n digit entries of `scalars` by bucket (bucket_bits bits of bucket index;
// per-window layout: window bits included).  The result (BucketOrder): the key/value arrays
// holding it (two of the lane's four entry buffers), the bucket starts (bucket b =
// [bstart[b], bstart[b+1]), b < 2^bucket_bits) and the shift from key to bucket; *valid =
// number of entries (non-zero digits).
//
// Three stages around the sort's one host wait (the last pass's tile-total readback):
// bucket_sort_begin queues pass 1, bucket_sort_passes the passes up to that readback, and
// bucket_sort_finish waits for it and queues the rest.  A pair of MSMs calls begin(a), begin(b),
// passes(a), passes(b), finish(a), finish(b): lane b's pass 1 is queued after ~5 host calls
// instead of lane a's ~20 (0.35 ms of launch overhead on the critical lane), and each lane's
// last pass starts as soon as ITS readback lands (a single host wait would hold lane a's last
// pass behind lane b's first two passes: ~1.7 ms of an idle lane per 2^24 opening pair).
void bucket_sort_begin(MsmLane &ln, const SortInput &in, size_t n, int c, int W, bool shared, uint32_t stride,
                       int bucket_bits, uint32_t *valid, BucketSortJob &J) {
  hipStream_t st = ln.stream;
  const size_t E = (size_t)W * n;
  if (E >= ((size_t)1 << 32)) throw Error(TNS_ERR_COMMITMENT, "MSM too large for one bucket sort");
  if (W > BS_TILE) throw Error(TNS_ERR_COMMITMENT, "too many MSM windows");
  J = BucketSortJob();
  J.ln = &ln;
  J.valid = valid;
  J.E = E;
  J.bucket_bits = bucket_bits;
  uint32_t **K = J.K, **V = J.V;
  K[0] = (uint32_t *)ln.ws[0].ensure(sizeof(uint32_t) * E);
  K[1] = (uint32_t *)ln.ws[2].ensure(sizeof(uint32_t) * E);
  V[0] = (uint32_t *)ln.ws[1].ensure(sizeof(uint32_t) * E);
  V[1] = (uint32_t *)ln.ws[3].ensure(sizeof(uint32_t) * E);
  DigitArgs A{in.fr, n, 0, c, W, 0, shared, stride, in.mont, in.u64, in.n_u64};
  if (shared)
    while ((1 << A.wb) < W) A.wb++;
  J.wb = A.wb;
  const int keybits = bucket_bits + A.wb;
  const int npass = std::max(1, (keybits + BS_MAXBITS - 1) / BS_MAXBITS);
  int *bits = J.bits;
  // the last pass sorts LDS-sized segments by BS_MAXBITS bits; the passes before it split the
  // remaining bits evenly (25-bit keys: 8, 8, 9 -- pass 2 with 256 instead of 512 bins writes
  // 128-byte runs: 1.21 -> 1.02 ms at 2^24)
  bits[npass - 1] = std::min(keybits, BS_MAXBITS);
  // packed tail: the second-to-last pass writes (last-pass key bits, sign, point index) as one
  // word when they fit (n <= 2^22 with a 9-bit last pass).  (A 7-bit last pass for 2^24 points,
  // 9, 9, 7, measured slower: it moved the cost into 512-bin passes, +3.3 ms of sort per C4 step
  // against -0.8 ms of reads.)  Values-only last pass (vo): whenever there is more than one pass --
  // the accumulation reads no keys (C4: k_accumulate 9.10 -> 8.8 ms).
  int ibits = 1;
  while (((size_t)1 << ibits) < n) ibits++;
  J.vo = npass >= 2;
  // (unpack_value reads the window index from the low wb bits of the last pass's L key bits: L >= wb)
  J.pk = J.vo && npass >= 3 && bits[npass - 1] + ibits + 1 <= 32 && bits[npass - 1] >= J.wb;
  for (int p = 0, rest = keybits - bits[npass - 1]; p < npass - 1; p++) {
    bits[p] = (rest + (npass - 2 - p)) / (npass - 1 - p);
    rest -= bits[p];
  }
  J.ibits = ibits;
  J.shared = shared;
  J.stride = stride;
  // key formats between passes: 2-byte keys into the last pass (its <= 9 key bits; C4 openings:
  // pass 2 -> 3, sort kernels -0.6 ms per step, profiles/r03_ab_sort_k16.txt), 4-byte keys elsewhere
  for (int p = 0, rest = keybits; p < npass - 1; p++) {
    rest -= bits[p];
    J.kf[p] = J.vo && p == npass - 2 && rest <= 16 ? KF_U16 : KF_U32;
  }
  if (J.pk) J.kf[npass - 2] = KF_U32;  // the packed words (pack_entry) are 4-byte
  int shift = keybits - bits[0];

  // pass 1: scalars -> bins of the top bits[0] key bits (a compile-time plan's kernels when there
  // is one for this window plan, else the runtime-plan kernels)
  const int tile1 = BS_TILE;
  const Pass1Plan *ct = nullptr;
  for (const Pass1Plan &p : kPass1Plans)
    if (p.tile == tile1 && p.c == c && p.W == W) ct = &p;
  if ((size_t)tile1 < (size_t)W) throw Error(TNS_ERR_INVALID_PARAMETERS, "bucket sort: more windows than a pass-1 tile holds");
  A.spb = (size_t)tile1 / W;
  if (ct) A.spb = std::min(A.spb, (size_t)BS_BLOCK * ct->spt);
  const size_t T1 = (n + A.spb - 1) / A.spb;
  int nb = 1 << bits[0];
  const Pass1Geom pg = pass1_geom(n, c, W, shared, bucket_bits);
  if (pg.bits0 != bits[0] || pg.T1 != T1 || pg.ct != ct || pg.shift != shift)
    throw Error(TNS_ERR_DEVICE, "bucket sort: pass-1 geometry mismatch");
  const size_t max_seg = (size_t)1 << keybits;
  uint32_t **seg = J.seg;
  seg[0] = (uint32_t *)ln.ws[10].ensure(sizeof(uint32_t) * (max_seg + 1));
  seg[1] = (uint32_t *)ln.ws[11].ensure(sizeof(uint32_t) * (max_seg + 1));
  const size_t tmin = 4096;  // the smallest pass tile
  const size_t max_tiles = (E + tmin - 1) / tmin + (max_seg >> bits[npass - 1]) + 1;
  const size_t cnt_len = std::max((size_t)nb * T1, (size_t)BS_MAXBINS * max_tiles) + 1;
  const bool pre = in.precounted && ct && in.pre_shared == shared && in.pre_c == c && in.pre_W == W &&
                   ln.ws[12].p == in.precounted && ln.ws[12].bytes >= sizeof(uint32_t) * cnt_len;
  uint32_t *counts = J.counts = (uint32_t *)ln.ws[12].ensure(sizeof(uint32_t) * cnt_len);
  uint32_t *offs = J.offs = (uint32_t *)ln.ws[13].ensure(sizeof(uint32_t) * cnt_len);
  if (!pre) {  // (precounted: quotient2_count_dev wrote them)
    if (ct) ct->count<<<(unsigned)T1, BS_BLOCK, 0, st>>>(A, shift, nb, T1, counts, nullptr, nullptr);
    else k_bs_count1<<<(unsigned)T1, BS_BLOCK, 0, st>>>(A, shift, nb, T1, counts);
    TNS_LAUNCH_CHECK();
  }
  exclusive_scan(st, ln.ws[9], counts, offs, (size_t)nb * T1 + 1);
  const int kf1 = npass > 1 ? J.kf[0] : KF_U32;
  if (ct) ct->scatter<<<(unsigned)T1, BS_BLOCK, 0, st>>>(A, shift, nb, T1, offs, kf1, K[0], V[0]);
  else k_bs_scatter1<BS_TILE><<<(unsigned)T1, BS_BLOCK, 0, st>>>(A, shift, nb, T1, offs, kf1, K[0], V[0]);
  TNS_LAUNCH_CHECK();
  k_bs_segs1<<<1, 256, 0, st>>>(offs, nb, T1, seg[0], valid);
  TNS_LAUNCH_CHECK();

  J.S = nb;
  J.cur = 0;
  J.tcount = (uint32_t *)ln.ws[14].ensure(sizeof(uint32_t) * 2 * (max_seg + 1));
  J.tbase = J.tcount + (max_seg + 1);
  J.desc = (uint32_t *)ln.ws[15].ensure(sizeof(uint32_t) * max_tiles);
  J.mcount = (uint32_t *)ln.ws[17].ensure(sizeof(uint32_t) * 2 * (max_seg + 1));
  J.mbase = J.mcount + (max_seg + 1);
  J.npass = npass;
  J.shift = shift;
  J.keybits = keybits;
}

// passes 2 .. up to the last pass's readback (queued on the lane; no host wait)
void bucket_sort_passes(BucketSortJob &J) {
  MsmLane &ln = *J.ln;
  hipStream_t st = ln.stream;
  const int npass = J.npass, keybits = J.keybits, *bits = J.bits;
  const size_t E = J.E;
  uint32_t **seg = J.seg;
  for (int p = 1; p < npass; p++) {
    J.p = p;
    J.nb = 1 << bits[p];
    J.shift -= bits[p];
    // 8192-entry tiles, except a last pass whose segments average <= 3584 entries (4096: the
    // one-tile segments fill it, and half the LDS doubles the blocks per CU -- pass 3 of a 2^24
    // opening MSM 1.02 -> 0.61 ms, profiles/r02_ab_sort_tiles.txt)
    const int tile = (p == npass - 1 && (E >> (keybits - bits[p])) <= 3584) ? 4096 : BS_TILE;
    J.tile = tile;
    // In the last pass most segments fit one tile and rank locally; only segments of >= 2
    // tiles need the histogram pass and the global scan, so their counts get a compact layout,
    // sized from a readback of the tile totals (the top window's narrow digits make the
    // low-magnitude buckets' segments multi-tile).  All one-tile: no geometry at all (at 2^24
    // the full layout's histograms and scan over 512 bins x every tile took 0.34 ms).
    J.last = p == npass - 1;
    if (J.S + 1 <= SCAN_SMALL) {  // the tile geometry in one launch (k_bs_geom)
      uint32_t *pub = nullptr, *flag = nullptr, seq = 0;
      if (J.last) lane_publish_slot(ln, LANE_SLOT_SORT, &pub, &flag, &seq);
      k_bs_geom<<<1, ONE_BLOCK, 0, st>>>(seg[J.cur], J.S, (uint32_t)tile, J.tbase, J.last ? J.mbase : nullptr, J.valid,
                                    pub, flag, seq);
      TNS_LAUNCH_CHECK();
      if (J.last) {
        J.pending = true;
        return;
      }
      bucket_sort_pass_rest(J, false);
      continue;
    }
    k_bs_tiles<<<grid_for(J.S + 1, 256), 256, 0, st>>>(seg[J.cur], J.S, (uint32_t)tile, J.tcount,
                                                         J.last ? J.mcount : nullptr);
    TNS_LAUNCH_CHECK();
    exclusive_scan(st, ln.ws[9], J.tcount, J.tbase, J.S + 1);
    if (J.last) {  // the readback; pass_rest runs after bucket_sort_finish's wait
      exclusive_scan(st, ln.ws[9], J.mcount, J.mbase, J.S + 1);
      // (with the entry count k_bs_segs1 wrote: the accumulation sizes its chunks from it)
      const void *src[3] = {J.tbase + J.S, J.mbase + J.S, J.valid};
      const size_t by[3] = {4, 4, 4};
      lane_publish(ln, LANE_SLOT_SORT, 3, src, by);
      J.pending = true;
      return;
    }
    bucket_sort_pass_rest(J, false);
  }
}

// the rest of pass (J.nb, J.shift, J.tile) after its tile counts: geometry, histograms, scan,
// scatter, next segment starts.  readback: the last pass, whose tile totals are in host2.
void bucket_sort_pass_rest(BucketSortJob &J, bool readback) {
  MsmLane &ln = *J.ln;
  hipStream_t st = ln.stream;
  const int nb = J.nb, tile = J.tile, cur = J.cur;
  const size_t S = J.S;
  int ident = 0;
  const uint32_t *mb = nullptr;
  size_t tiles_bound = (J.E + tile - 1) / tile + S, scan_len = (size_t)nb * tiles_bound + 1;
  if (readback) {
    const uint32_t *h = (const uint32_t *)J.readback;
    ident = h[1] == 0;
    tiles_bound = ident ? S : h[0];
    mb = J.mbase;
    scan_len = (size_t)nb * h[1] + 1;
  }
  if (!ident) {
    k_bs_desc<<<grid_for(tiles_bound, 256, 4096), 256, 0, st>>>(J.tbase, S, J.desc);
    TNS_LAUNCH_CHECK();
  }
  // packed tail: pass npass - 2 writes packed words, the last pass bins them by their top bits
  const int pk = J.pk ? (J.p == J.npass - 2 ? 1 : J.p == J.npass - 1 ? 2 : 0) : J.vo && J.p == J.npass - 1 ? 3 : 0;
  const PackArgs PA{J.ibits, J.bits[J.npass - 1], J.wb, J.shared ? 1 : 0, J.stride};
  const int kin = J.kf[J.p - 1], kout = J.p < J.npass - 1 ? J.kf[J.p] : KF_U32;
  PassGeom G{J.seg[cur], J.tbase, J.desc, pk == 2 ? J.ibits + 1 : J.shift, nb, (uint32_t)nb - 1, ident, mb, kin,
             pk == 0 ? kout : KF_U32};
  uint32_t *counts = J.counts, *offs = J.offs;
  if (!ident) {
    if (mb) TNS_HIP(hipMemsetAsync(counts + (scan_len - 1), 0, sizeof(uint32_t), st));  // the scan's total slot
    if (tile == 4096) k_bs_count<4096><<<(unsigned)tiles_bound, BS_BLOCK, 0, st>>>(G, S, tiles_bound, J.K[cur], counts);
    else k_bs_count<BS_TILE><<<(unsigned)tiles_bound, BS_BLOCK, 0, st>>>(G, S, tiles_bound, J.K[cur], counts);
    TNS_LAUNCH_CHECK();
    exclusive_scan(st, ln.ws[9], counts, offs, scan_len);
  }
  {
    auto *kern = tile == 4096 ? (pk == 0   ? k_bs_scatter<4096, 0>
                                 : pk == 1 ? k_bs_scatter<4096, 1>
                                 : pk == 2 ? k_bs_scatter<4096, 2>
                                           : k_bs_scatter<4096, 3>)
                              : (pk == 0   ? k_bs_scatter<BS_TILE, 0>
                                 : pk == 1 ? k_bs_scatter<BS_TILE, 1>
                                 : pk == 2 ? k_bs_scatter<BS_TILE, 2>
                                           : k_bs_scatter<BS_TILE, 3>);
    kern<<<(unsigned)tiles_bound, BS_BLOCK, 0, st>>>(G, S, offs, J.K[cur], J.V[cur], J.K[cur ^ 1], J.V[cur ^ 1],
                                                     J.seg[cur ^ 1], PA);
  }
  TNS_LAUNCH_CHECK();
  k_bs_segs<<<grid_for(S * nb + 1, 256), 256, 0, st>>>(G, S, offs, J.seg[cur ^ 1]);
  TNS_LAUNCH_CHECK();
  J.cur ^= 1;
  J.S *= nb;
}

BucketOrder bucket_sort_finish(BucketSortJob &J) {
  MsmLane &ln = *J.ln;
  size_t entries = SIZE_MAX;  // unknown without the readback
  if (J.pending) {  // the last pass's tile totals
    J.readback = lane_wait(ln, LANE_SLOT_SORT);
    J.pending = false;
    entries = ((const uint32_t *)J.readback)[2];
    bucket_sort_pass_rest(J, true);
  }
  uint32_t *bstart = J.seg[J.cur];
  if (J.wb) {  // (bucket, window) segments -> bucket starts
    bstart = J.seg[J.cur ^ 1];
    const size_t nbk = (size_t)1 << J.bucket_bits;
    k_bs_bucket_starts<<<grid_for(nbk + 1, 256), 256, 0, ln.stream>>>(J.seg[J.cur], nbk, J.wb, bstart);
    TNS_LAUNCH_CHECK();
  }
  return BucketOrder{J.vo ? nullptr : J.K[J.cur], J.V[J.cur], bstart, J.wb, entries};
}

// The opening quotients (lagrange.hip k_node_quotient2_canon<true>) fused with both sorts' pass-1
// histograms (k_bs_count1_ct): one block per pass-1 tile of spb nodes; the block writes q0 / q1,
// their bit lengths, and each quotient's digits' bins into two LDS histograms.
template <int C, int W>
__global__ void __launch_bounds__(BS_BLOCK) k_quotient2_count1(const Fr *__restrict__ y0, const Fr *__restrict__ y1,
                                                               Fr v0, Fr v1, size_t n, const Fr *invs,
                                                               Fr *__restrict__ q0, Fr *q1, unsigned *__restrict__ bits,
                                                               size_t spb, int wb, int shift, int nbins, size_t T1,
                                                               uint32_t *__restrict__ counts0,
                                                               uint32_t *__restrict__ counts1) {
  __shared__ uint32_t h0[BS_MAXBINS], h1[BS_MAXBINS];
  for (int d = threadIdx.x; d < nbins; d += BS_BLOCK) h0[d] = h1[d] = 0;
  __syncthreads();
  DigitArgs A{};
  A.shared = true;
  A.wb = wb;
  const size_t tile = blockIdx.x, a = tile * spb, b = min(n, a + spb);
  unsigned b0 = 0, b1 = 0;
  for (size_t i = a + threadIdx.x; i < b; i += BS_BLOCK) {
    const Fr iv = invs[i];  // (q1 may be invs itself: each i is read, then written, by one thread)
    const Fr c0 = mul(sub(v0, y0[i]), iv), c1 = mul(sub(v1, y1[i]), iv);
    q0[i] = c0;
    q1[i] = c1;
    b0 = max(b0, fr_bit_length(c0));
    b1 = max(b1, fr_bit_length(c1));
    scalar_digits_ct<C, W>(c0, A, [&](int, uint32_t key, bool) { atomicAdd(&h0[key >> shift], 1u); });
    scalar_digits_ct<C, W>(c1, A, [&](int, uint32_t key, bool) { atomicAdd(&h1[key >> shift], 1u); });
  }
  __syncthreads();
  for (int d = threadIdx.x; d < nbins; d += BS_BLOCK) {
    counts0[(size_t)d * T1 + tile] = h0[d];
    counts1[(size_t)d * T1 + tile] = h1[d];
  }
  if (tile == 0 && threadIdx.x == 0) counts0[(size_t)nbins * T1] = counts1[(size_t)nbins * T1] = 0;
  block_atomic_max2(b0, b1, bits, bits + 1);
}

bool quotient2_count_dev(Ctx *c, const Fr *y0, const Fr *y1, size_t n, const Fr &v0, const Fr &v1, const Fr *inv,
                         Fr *q0, Fr *q1, unsigned *bits, int cw, int W, const uint32_t *counts_out[2]) {
  if (cw != 22 || W != 12) return false;  // (the openings' table plan at 2^21..2^26 nodes; else unfused)
  const Pass1Geom g = pass1_geom(n, cw, W, true, cw - 1);
  if (!g.ct || g.npass < 2) return false;
  uint32_t *cnt[2];
  for (int k = 0; k < 2; k++) cnt[k] = (uint32_t *)c->lanes[k].ws[12].ensure(sizeof(uint32_t) * g.cnt_len);
  TNS_PROF(c, "open_scan", 32.0 * 5 * n);
  TNS_HIP(hipMemsetAsync(bits, 0, 2 * sizeof(unsigned), c->stream));
  k_quotient2_count1<22, 12><<<(unsigned)g.T1, BS_BLOCK, 0, c->stream>>>(y0, y1, v0, v1, n, inv, q0, q1, bits, g.spb, g.wb,
                                                                          g.shift, g.nb, g.T1, cnt[0], cnt[1]);
  TNS_LAUNCH_CHECK();
  counts_out[0] = cnt[0];
  counts_out[1] = cnt[1];
  return true;
}

bool bucket_sort_precount_bits(MsmLane &ln, const Fr *scalars, size_t n, int c, int W, bool shared, int bucket_bits,
                               unsigned *bits, SortInput &in, bool want_low64) {
  const Pass1Geom g = pass1_geom(n, c, W, shared, bucket_bits);
  if (!g.ct) return false;
  uint32_t *counts = (uint32_t *)ln.ws[12].ensure(sizeof(uint32_t) * g.cnt_len);
  uint64_t *low = want_low64 ? (uint64_t *)ln.ws[18].ensure(sizeof(uint64_t) * n) : nullptr;
  DigitArgs A{scalars, n, g.spb, c, W, g.wb, shared, 0u, true, nullptr, 0};
  g.ct->count<<<(unsigned)g.T1, BS_BLOCK, 0, ln.stream>>>(A, g.shift, g.nb, g.T1, counts, bits, low);
  TNS_LAUNCH_CHECK();
  in.low64 = low;
  in.precounted = counts;
  in.pre_c = c;
  in.pre_W = W;
  in.pre_shared = shared;
  return true;
}

BucketOrder bucket_sort_dev(MsmLane &ln, const SortInput &in, size_t n, int c, int W, bool shared, uint32_t stride,
                            int bucket_bits, uint32_t *valid) {
  BucketSortJob J;
  bucket_sort_begin(ln, in, n, c, W, shared, stride, bucket_bits, valid, J);
  bucket_sort_passes(J);
  return bucket_sort_finish(J);
}

}  // namespace tns
