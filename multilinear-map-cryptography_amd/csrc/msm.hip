// msm.hip -- BN254 G1 multi-scalar multiplication (Pippenger, signed windows).
//
// Replaces KZGCommitment::commit's per-term scalar multiplications
// (src/commitments.rs:173-177): C = sum_i c_i * g1_powers[i].  The group element
// is unique, so any correct algorithm reproduces it exactly.
//
// Two bucket layouts share one pipeline:
//  * per-window: W windows of c bits, W * 2^(c-1) buckets, windows combined by Horner;
//  * shared (fixed bases: the SRS and its Lagrange bases never change): a precomputed
//    table T[j n + i] = 2^(c j) P_i turns window j's digit of scalar i into a digit of
//    point T[j n + i], so all windows land in ONE set of 2^(c-1) buckets -- the bucket
//    reduction runs once instead of W times, no Horner doublings remain, and a wider c
//    (fewer windows, fewer bucket additions) becomes affordable.
//
// Pipeline (per MSM lane stream):
//  0. k_scalar_bits: bit length of the largest scalar -> windows above it are skipped
//     (trace commitments -- addresses, small values, flags -- are narrow).
//  1.-3. the bucket order (bucket_sort.hip): the signed c-bit digits are computed inside the
//     first pass of a hand-written MSD counting sort (no digit array, zero digits never enter it);
//     its last pass writes the point indices | sign<<31 alone and the bucket starts.
//  4. k_accumulate: load-balanced -- each thread owns acc_k consecutive sorted entries
//     and XYZZ-madds the (possibly negated) affine points run by run; runs that cross a
//     chunk boundary leave a head/tail partial; k_bucket_fixup completes those buckets (heavy buckets'
//     chunk heads through FIX_FAN-ary level sums, so no thread walks a long run).
//  5. k_reduce_level: per group of L buckets of a window, running sums
//     T_g = sum_{j in g} (j - a + 1) B_j and S_g = sum_{j in g} B_j; then
//     sum_j (j+1) B_j = sum_g T_g + L sum_g g S_g, and sum_g g S_g = sum_b 2^b M_b with
//     M_b the sum of the S_g whose index has bit b set: k_masked_sums + chunked sums
//     (short dependency chains -- single-thread point-add chains are the slow part).
//  6. host: per-window Horner (per-window layout) or nothing (shared layout).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <memory>
#include <cstdlib>
#include <vector>

#include "common.hpp"

namespace tns {

constexpr int RED_L = 16;  // running-sum group size of the bucket reduction

struct MsmPlan {
  bool shared = false;  // fixed-base shared-bucket layout
  int c = 0, W = 0, wbits = 0;
  uint32_t sentinel = 0;
  int end_bit = 0;
  size_t nb = 0;      // buckets in total
  int Wr = 0;         // bucket sets (windows) to reduce: W (per-window) or 1 (shared)
  size_t half = 0;    // buckets per set, 2^(c-1)
  size_t stride = 0;  // shared: table stride n_table (value = j * stride + i)
};

// signed-digit windows of c bits for `bits`-bit scalars: the top window's raw value
// < 2^(bits - c(W-1)) must stay <= 2^(c-1) so that it never carries out
static int windows_for(int bits, int c) {
  int W = (bits + c - 1) / c;
  if (bits - c * (W - 1) > c - 1) W++;
  return W;
}

// bucket additions + ~3 additions per bucket in the reduction
static double plan_cost(size_t n, int W, int c, int sets) {
  return (double)W * (double)n + 3.0 * sets * (double)((size_t)1 << (c - 1));
}

// w1max > cmax: scalars of up to w1max - 1 bits may also take one window of bits + 1 (no
// second window for the signed digits' carry, e.g. 22-bit trace addresses: n additions
// instead of 2n, and no thousands-deep buckets)
// tie: a window must cost below tie x the best smaller one to be taken (0.98: near-ties go to the
// smaller window, less bucket memory)
static int best_window(size_t n, int bits, int cmax, bool shared, int w1max = 0, double tie = 0.98) {
  int lg = 0;
  while (((size_t)1 << lg) < n) lg++;
  double best = 1e300;
  int bc = 4;
  for (int c = 4; c <= cmax && c <= lg + 2; c++) {
    const int W = windows_for(bits, c);
    const double cost = plan_cost(n, W, c, shared ? 1 : W);
    if (cost < best * tie) {
      best = cost;
      bc = c;
    }
  }
  const int c1 = bits + 1;
  if (c1 > cmax && c1 <= w1max && c1 <= lg + 2 && plan_cost(n, 1, c1, 1) < best * tie) bc = c1;
  return bc;
}

static void finish_plan(MsmPlan &p) {
  p.half = (size_t)1 << (p.c - 1);
  if (p.shared) {
    p.wbits = 0;
    p.Wr = 1;
  } else {
    p.wbits = 0;
    while ((1 << p.wbits) < p.W) p.wbits++;
    p.Wr = p.W;
  }
  p.end_bit = p.wbits + (p.c - 1) + 1;
  p.sentinel = 1u << (p.wbits + p.c - 1);
  p.nb = (size_t)p.Wr * p.half;
}

// *bits = max over i of bitlen(canonical scalar_i); canon (optional) = the canonical scalars
// (the bucket sort canonicalises Montgomery scalars itself, so the MSMs pass none)
__global__ void __launch_bounds__(256) k_scalar_bits(const Fr *__restrict__ scalars, size_t n,
                                                     unsigned *__restrict__ bits, Fr *__restrict__ canon) {
  unsigned b = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    Fr k = from_mont(scalars[i]);
    if (canon) canon[i] = k;
    b = max(b, fr_bit_length(k));
  }
  block_atomic_max2(b, 0u, bits, nullptr);
}

// the accumulation's point gather
__device__ __forceinline__ G1Affine load_point(const G1Affine *__restrict__ pts, uint32_t i) { return pts[i]; }

struct HeadTail {
  G1Xyzz head, tail;
};

// the bucket holding sorted entry p < valid: the largest k with bstart[k] <= p (bstart is
// non-decreasing, bstart[0] = 0, bstart[nb] = valid; empty buckets repeat their successor's start)
__device__ __forceinline__ uint32_t bucket_of(const uint32_t *__restrict__ bstart, size_t nb, size_t p) {
  size_t lo = 0, hi = nb;
  while (hi - lo > 1) {
    const size_t mid = (lo + hi) >> 1;
    if (bstart[mid] <= p) lo = mid;
    else hi = mid;
  }
  return (uint32_t)lo;
}

constexpr int FIX_FAN = 8;  // short peel chains: single-thread add chains are latency-bound

// keys == nullptr (values-only sort tail): a chunk finds its first bucket by a binary search of the
// bucket starts and every later run boundary from the next start -- no key per entry.
// KEYS (a template parameter, so the default values-only sort's variant carries none of the key
// path's registers): the sort left a key per entry (else the runs come from the bucket starts)
template <bool KEYS>
__global__ void __launch_bounds__(256) k_accumulate(const uint32_t *__restrict__ keys,
                                                    const uint32_t *__restrict__ vals,
                                                    const uint32_t *__restrict__ valid_p,
                                                    const G1Affine *__restrict__ pts,
                                                    G1Xyzz *__restrict__ buckets,
                                                    HeadTail *__restrict__ ht, size_t nchunks, int ks,
                                                    int acc_k, const uint32_t *__restrict__ bstart, size_t nb,
                                                    uint2 *__restrict__ cbk, uint32_t *__restrict__ spans) {
  // entry positions are 32-bit (a sort holds < 2^31 entries, msm_launch_sort): one VGPR each
  const uint32_t valid = *valid_p;
  bool crossed = false;  // this thread left a head or tail partial (k_fix_level / k_bucket_fixup work)
  bool grouped = false;  // ... and a level-1 group of 8 chunks lies inside one bucket (k_fix_level's)
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < nchunks;
       t += (size_t)gridDim.x * blockDim.x) {
    const uint32_t a = (uint32_t)t * (uint32_t)acc_k;
    uint32_t fb = 0xffffffffu, lb = 0xfffffffeu;  // the chunk's first / last bucket (none past valid)
    if (a < valid) {
    const uint32_t b = a + acc_k < valid ? a + acc_k : valid;
    // a run is a head (it began before this chunk) iff it is the chunk's first run and entry
    // a - 1 has its bucket, a tail (it goes on after the chunk) iff it is the last run and entry
    // b has its bucket: two key loads per chunk instead of the run's bounds at every flush.
    // Flushed sums stay in the lazy domain [0, 2M): the fixup and the reduction add them lazily.
    uint32_t cur, after;
    bool head_run;
    uint32_t nxt = 0;  // (no keys) the start of the bucket after `cur`
    if (KEYS) {
      cur = keys[a] >> ks;
      head_run = a > 0 && (keys[a - 1] >> ks) == cur;
      after = b < valid ? keys[b] >> ks : 0xffffffffu;
    } else {
      cur = bucket_of(bstart, nb, a);
      head_run = bstart[cur] < a;
      nxt = bstart[cur + 1];
      after = 0xffffffffu;
    }
    bool first = true;
    const uint32_t first_bucket = cur;
    G1Xyzz acc = G1Xyzz::inf();
    for (uint32_t p = a;; p++) {
      const bool brk = KEYS ? p >= b || (keys[p] >> ks) != cur : p >= b || p >= nxt;
      if (brk) {  // flush the run of bucket `cur`
        const bool tail = KEYS ? after == cur : nxt > b;
        if (first && head_run) ht[t].head = acc;
        else if (p >= b && tail) ht[t].tail = acc;
        else buckets[cur] = acc;
        crossed |= (first && head_run) || (p >= b && tail);
        if (p >= b) {
          cbk[t] = make_uint2(first_bucket, cur);  // the buckets of entries a and b - 1 (k_fix_level)
          fb = first_bucket;
          lb = cur;
          break;
        }
        first = false;
        if (KEYS) {
          cur = keys[p] >> ks;
        } else {
          do {  // skip empty buckets
            cur++;
            nxt = bstart[cur + 1];
          } while (nxt <= p);
        }
        acc = G1Xyzz::inf();
      }
      // (gathering entry p + 1 ahead of this addition measured no faster: 39.48 vs 39.46 ms of
      // accumulation per C4 step -- three waves per SIMD hide the gather)
      const uint32_t v = vals[p];
      G1Affine q = load_point(pts, v & 0x7fffffffu);
      // -y = M - y (y canonical); the identity (0, 0) keeps y = 0
      const Fq ny = const_minus_dev<FqCfg, false>(q.y);
      const bool negy = (v >> 31) && !q.y.is_zero();
#pragma unroll
      for (int l = 0; l < 8; l++) q.y.v[l] = negy ? ny.v[l] : q.y.v[l];
      acc = xyzz_madd_lazy(acc, q);
    }
    }
    // k_fix_level's level-1 test for the group of chunks t .. t + 7 (t a multiple of 8: lane 8k):
    // the first chunk's first bucket is the last chunk's last (every lane of the wave shuffles)
    const uint32_t lb7 = __shfl_down(lb, 7, FIX_FAN);
    grouped |= (threadIdx.x & (FIX_FAN - 1)) == 0 && t + FIX_FAN - 1 < nchunks && fb == lb7;
  }
  // two flags per MSM: no run crossed a chunk (the 22-bit address commitment at C4: every bucket's
  // four entries inside one chunk) -> nothing to fix up; no 8-chunk group inside one bucket (any
  // uniform scalars: the openings, C2) -> no fix level has a group to sum
  const uint32_t f = (__any(crossed) ? 1u : 0u) | (__any(grouped) ? 2u : 0u);  // (every lane votes)
  if (f && (threadIdx.x & 63) == 0) atomicOr(spans, f);
}

// Heavy buckets (skewed scalars: repeated values, small ranges) span many chunks; their
// chunk heads are summed through a FIX_FAN-ary hierarchy so no thread walks a long run.
// Level l >= 1, group g covers chunks [g F^l, (g+1) F^l) (F = FIX_FAN); its sum is formed only when
// every sorted entry of those chunks has one key (then every head in it is a full-chunk
// sum of that bucket); other groups are never read.
constexpr int FIX_LEVELS = 8;
struct FixLevels {
  G1Xyzz *lv[FIX_LEVELS + 1];  // lv[l] for l >= 1 (the level-0 heads live in ht)
  size_t len[FIX_LEVELS + 1];
  int n;                        // levels built (0: none)
};

// FIX_FAN consecutive lanes per group: lane j loads item j and the group's sum is an xor butterfly
// over those lanes (3 dependent additions instead of one thread's chain of 7: the narrow value
// commitment's heavy buckets fill thousands of groups and this level ran at half a wave per SIMD)
static_assert(FIX_FAN == 8, "k_fix_level's butterfly assumes 8 lanes per group");
// one MSM's level-l groups (blockIdx.y picks the MSM: a pair's two tails run as one launch)
struct FixLevelSet {
  const uint32_t *valid;
  const HeadTail *ht;
  const G1Xyzz *below;
  G1Xyzz *out;
  const uint2 *cbk;
  size_t n_groups;  // 0: this MSM has no level l
  int acc_k;
};
struct FixLevelArgs {
  FixLevelSet s[2];
};
__global__ void __launch_bounds__(256) k_fix_level(FixLevelArgs A, int level) {
  const FixLevelSet &S = A.s[blockIdx.y];
  const size_t n_groups = S.n_groups;
  // (valid[1] bit 1: some 8-chunk group lies inside one bucket, k_accumulate; a group of any
  // higher level is made of such groups)
  if (!n_groups || !(S.valid[1] & 2u)) return;
  const size_t valid = *S.valid;
  const int acc_k = S.acc_k;
  const int j = threadIdx.x & (FIX_FAN - 1);
  const size_t stride = (size_t)gridDim.x * blockDim.x / FIX_FAN;
  // group-uniform trip count (blockDim.x is a multiple of FIX_FAN): the 8 lanes of a group stay together
  for (size_t g = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) / FIX_FAN; g < n_groups; g += stride) {
    size_t span = (size_t)acc_k;
    for (int l = 0; l < level; l++) span *= FIX_FAN;
    const size_t a = g * span, b = a + span;  // entries covered
    // every entry of [a, b) in one bucket: the bucket of entry a (that chunk's first) is the bucket
    // of entry b - 1 (the last chunk's last), as k_accumulate recorded them
    const bool uniform = b <= valid && S.cbk[a / acc_k].x == S.cbk[(b - 1) / acc_k].y;
    // a wave whose 8 groups all span several buckets has nothing to sum (those sums are never
    // read): skip its butterfly -- most of a narrow commitment's groups (the 22-bit address MSM:
    // ~4 entries a bucket) are such
    if (!__any(uniform)) continue;
    G1Xyzz acc = G1Xyzz::inf();
    if (uniform) acc = level == 1 ? S.ht[g * FIX_FAN + j].head : S.below[g * FIX_FAN + j];
    for (int off = FIX_FAN / 2; off > 0; off >>= 1) {  // every lane of the wave takes part
      G1Xyzz o;
      const uint32_t *pa = reinterpret_cast<const uint32_t *>(&acc);
      uint32_t *po = reinterpret_cast<uint32_t *>(&o);
#pragma unroll
      for (int q = 0; q < (int)(sizeof(G1Xyzz) / 4); q++) po[q] = __shfl_xor(pa[q], off);
      if (uniform) acc = xyzz_add_lazy(acc, o);
    }
    if (uniform && j == 0) S.out[g] = acc;
  }
}

// bucket values: empty -> identity; a run inside one chunk is already in buckets[bk];
// a run across chunks tf < tl -> tail(tf) + heads of (tf, tl) (via the levels) + head(tl)
// Runs over more than FIX_WAVE_SPAN chunks are summed by the whole wave that meets them in
// k_bucket_fixup: a single thread's chain over their ~50+ items would be the tail of the whole
// MSM (a skewed input puts every entry in one bucket: Shout's identity lookups, 5.8 instead of
// 6.4 ms at 2^20).  Shorter runs stay one thread each -- thousands of moderately heavy buckets
// (the top window's narrow digits crowd the low ones) are cheaper so than as thousands of
// mostly idle wave passes next to the other lane's accumulation.
constexpr size_t FIX_WAVE_SPAN = 512;

// the items of a run across chunks tf < tl, in order: tail(tf), head(tl), then the inner heads
// (tf, tl), peeled to FIX_FAN-aligned ranges and climbing a level whenever both ends are aligned
struct FixItems {
  size_t tf, tl, lo, hi;
  int l, k;  // level, items produced so far
  __device__ FixItems(size_t f, size_t t) : tf(f), tl(t), lo(f + 1), hi(t), l(0), k(0) {}
  __device__ const G1Xyzz *next(const HeadTail *ht, const FixLevels &F) {
    if (k == 0) {
      k++;
      return &ht[tf].tail;
    }
    if (k == 1) {
      k++;
      return &ht[tl].head;
    }
    for (;;) {
      if (lo >= hi) return nullptr;
      const bool climb = l < F.n && hi - lo >= 2 * FIX_FAN;
      if (climb && lo % FIX_FAN == 0 && hi % FIX_FAN == 0) {
        lo /= FIX_FAN;
        hi /= FIX_FAN;
        l++;
        continue;
      }
      size_t i;
      if (!climb || lo % FIX_FAN) i = lo++;
      else i = --hi;  // lo aligned, hi not
      k++;
      return l == 0 ? &ht[i].head : &F.lv[l][i];
    }
  }
};

// the sum over the wave of every lane's acc, in every lane (xor butterfly: 6 dependent additions)
__device__ __forceinline__ G1Xyzz wave_sum_xyzz(G1Xyzz acc) {
  for (int off = 32; off > 0; off >>= 1) {
    G1Xyzz o;
    const uint32_t *pa = reinterpret_cast<const uint32_t *>(&acc);
    uint32_t *po = reinterpret_cast<uint32_t *>(&o);
#pragma unroll
    for (int q = 0; q < (int)(sizeof(G1Xyzz) / 4); q++) po[q] = __shfl_xor(pa[q], off);
    acc = xyzz_add_lazy(acc, o);
  }
  return acc;
}

// one MSM's buckets (blockIdx.y picks the MSM: a pair's two tails run as one launch)
struct FixupSet {
  const uint32_t *start, *end;
  const uint32_t *valid;  // [1]: some run crossed a chunk (else only the empty buckets need writing)
  const HeadTail *ht;
  FixLevels F;
  G1Xyzz *buckets;
  size_t nb;
  int acc_k;
};
struct FixupArgs {
  FixupSet s[2];
};
__global__ void __launch_bounds__(256) k_bucket_fixup(FixupArgs A) {
  const FixupSet &S = A.s[blockIdx.y];
  const uint32_t *__restrict__ start = S.start;
  const uint32_t *__restrict__ end = S.end;
  const HeadTail *__restrict__ ht = S.ht;
  const FixLevels &F = S.F;
  G1Xyzz *__restrict__ buckets = S.buckets;
  const size_t nb = S.nb;
  const int acc_k = S.acc_k;
  const int lane = threadIdx.x & 63;
  if (!S.valid[1]) {  // every run inside one chunk: k_accumulate wrote every non-empty bucket
    for (size_t bk = blockIdx.x * (size_t)blockDim.x + threadIdx.x; bk < nb; bk += (size_t)gridDim.x * blockDim.x)
      if (start[bk] == end[bk]) buckets[bk] = G1Xyzz::inf();
    return;
  }
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  // wave-uniform trip count: a wave meets its lanes' heavy runs together
  for (size_t base = blockIdx.x * (size_t)blockDim.x + (threadIdx.x & ~63u); base < nb; base += stride) {
    const size_t bk = base + lane;
    uint32_t s = 0, e = 0;
    if (bk < nb) {
      s = start[bk];
      e = end[bk];
    }
    const size_t tf = s / acc_k, tl = e > s ? (e - 1) / acc_k : tf;
    const bool heavy = bk < nb && tl - tf > FIX_WAVE_SPAN;
    // the wave's heavy runs, one at a time: lane j adds items j, j + 64, ..., then a butterfly
    for (uint64_t hm = __ballot(heavy); hm; hm &= hm - 1) {
      const int src = __ffsll((unsigned long long)hm) - 1;
      const size_t hf = __shfl((unsigned)tf, src), hl = __shfl((unsigned)tl, src);
      FixItems it(hf, hl);
      G1Xyzz acc = G1Xyzz::inf();
      const G1Xyzz *mine = nullptr;
      for (int k = 0;; k++) {  // the item sequence is the same in every lane: uniform control flow
        const G1Xyzz *item = it.next(ht, F);
        if (item && (k & 63) == lane) mine = item;
        if (!item || (k & 63) == 63) {  // a round of 64 items: every lane adds its own at once
          if (mine) acc = xyzz_add_lazy(acc, *mine);
          mine = nullptr;
          if (!item) break;
        }
      }
      acc = wave_sum_xyzz(acc);
      if (lane == src) buckets[bk] = acc;
    }
    if (bk >= nb || heavy) continue;
    if (s == e) {
      buckets[bk] = G1Xyzz::inf();
      continue;
    }
    if (tf == tl) continue;
    // one addition site: the items are head(tl), then the inner heads (tf, tl), peeled
    // to FIX_FAN-aligned ranges and climbing a level whenever both ends are aligned
    G1Xyzz acc = ht[tf].tail;
    size_t lo = tf + 1, hi = tl;
    int l = 0;
    bool pending_head = true;
    for (;;) {
      const G1Xyzz *item;
      if (pending_head) {
        item = &ht[tl].head;
        pending_head = false;
      } else {
        if (lo >= hi) break;
        const bool climb = l < F.n && hi - lo >= 2 * FIX_FAN;
        if (climb && lo % FIX_FAN == 0 && hi % FIX_FAN == 0) {
          lo /= FIX_FAN;
          hi /= FIX_FAN;
          l++;
          continue;
        }
        size_t i;
        if (!climb || lo % FIX_FAN) i = lo++;
        else i = --hi;  // lo aligned, hi not
        item = l == 0 ? &ht[i].head : &F.lv[l][i];
      }
      acc = xyzz_add_lazy(acc, *item);
    }
    buckets[bk] = acc;
  }
}

// one level over X (sets x n): groups of L; T = sum (j - a + 1) X_j, S = sum X_j
__global__ void __launch_bounds__(64) k_reduce_level(const G1Xyzz *__restrict__ X, int sets, size_t n, int L,
                                                     G1Xyzz *__restrict__ T, G1Xyzz *__restrict__ S) {
  const size_t groups = n / L;
  for (size_t id = blockIdx.x * (size_t)blockDim.x + threadIdx.x; id < (size_t)sets * groups;
       id += (size_t)gridDim.x * blockDim.x) {
    const size_t r = id / groups, g = id % groups;
    const G1Xyzz *x = X + r * n + g * L;
    G1Xyzz run = G1Xyzz::inf(), acc = G1Xyzz::inf();
    for (int j = L - 1; j >= 0; j--) {
      run = xyzz_add_lazy(run, x[j]);
      acc = xyzz_add_lazy(acc, run);
    }
    T[id] = acc;
    S[id] = run;
  }
}

// second level over the first level's (T, S) (sets x g1, groups of L1): per group h
//   u_h = sum T_g,  S2_h = sum S_g,  W_h = sum_j j S_{h L1 + j}  (the running sum added BEFORE
//   each element: no negation), and V_h = u_h + 2^lg0 W_h (lg0 doublings: L0 = 2^lg0).
// Then sum_g T_g + L0 sum_g g S_g = sum_h V_h + L0 L1 sum_h h S2_h, so the masked sums run over
// g1 / L1 groups with weight L0 L1.  Short chains (3 L1 additions + lg0 doublings) instead of the
// masked sums' ~nbits/2-fold re-reading of every S_g: C2's masked sums took 0.32 of its 2.3 ms.
__global__ void __launch_bounds__(64) k_reduce_level2(const G1Xyzz *__restrict__ T, const G1Xyzz *__restrict__ S,
                                                      int sets, size_t g1, int L1, int lg0,
                                                      G1Xyzz *__restrict__ V, G1Xyzz *__restrict__ S2) {
  const size_t groups = g1 / L1;
  for (size_t id = blockIdx.x * (size_t)blockDim.x + threadIdx.x; id < (size_t)sets * groups;
       id += (size_t)gridDim.x * blockDim.x) {
    const size_t r = id / groups, h = id % groups;
    const size_t base = r * g1 + h * L1;
    G1Xyzz run = G1Xyzz::inf(), w = G1Xyzz::inf(), u = G1Xyzz::inf();
    for (int j = L1 - 1; j >= 0; j--) {
      w = xyzz_add_lazy(w, run);  // + sum_{k > j} S_k: S_k counted k times in the end
      run = xyzz_add_lazy(run, S[base + j]);
      u = xyzz_add_lazy(u, T[base + j]);
    }
    w = xyzz_canon(w);
    for (int q = 0; q < lg0; q++) w = xyzz_dbl(w);
    V[id] = xyzz_add_lazy(u, w);
    S2[id] = run;
  }
}

// parts[(r specs + s) nch + ch], nch = g / (2 CH) chunks of CH items per spec s of set r:
//   s < nbits: the groups gi with bit s set, enumerated directly (the k-th is k with a one
//   inserted at bit s: every lane of a wave adds, no masked-off lanes);
//   s == nbits, nbits + 1: T over the lower / upper half of the groups
// wave_tree (nch a multiple of 64): the wave's 64 chunk sums are added in registers and only
// parts[id / 64] is written -- the two 8-way k_sum_chunks passes after it (each a chain of 8
// additions at low occupancy) become one 6-step butterfly
__global__ void __launch_bounds__(64) k_masked_sums(const G1Xyzz *__restrict__ T, const G1Xyzz *__restrict__ S,
                                                    int sets, size_t g, int nbits, int CH,
                                                    G1Xyzz *__restrict__ parts, bool wave_tree) {
  const int specs = nbits + 2;
  const size_t nch = g / (2 * (size_t)CH);
  for (size_t id = blockIdx.x * (size_t)blockDim.x + threadIdx.x; id < (size_t)sets * specs * nch;
       id += (size_t)gridDim.x * blockDim.x) {
    const size_t r = id / (specs * nch), rem = id % (specs * nch);
    const int sp = (int)(rem / nch);
    const size_t ch = rem % nch;
    G1Xyzz acc = G1Xyzz::inf();
    if (sp >= nbits) {
      const G1Xyzz *src = T + r * g + (size_t)(sp - nbits) * (g / 2);
      for (size_t k = ch * CH; k < ch * CH + CH; k++) acc = xyzz_add_lazy(acc, src[k]);
    } else {
      const G1Xyzz *src = S + r * g;
      const size_t lo_mask = ((size_t)1 << sp) - 1;
      for (size_t k = ch * CH; k < ch * CH + CH; k++)
        acc = xyzz_add_lazy(acc, src[((k & ~lo_mask) << 1) | ((size_t)1 << sp) | (k & lo_mask)]);
    }
    if (wave_tree) {  // the id range is a multiple of 64: every lane of the wave is here
      acc = wave_sum_xyzz(acc);
      if ((threadIdx.x & 63) == 0) parts[id >> 6] = acc;
    } else {
      parts[id] = acc;
    }
  }
}

// out[t] = sum of in[t*chunk .. (t+1)*chunk)
__global__ void __launch_bounds__(64) k_sum_chunks(const G1Xyzz *__restrict__ in, size_t n_out, int chunk,
                                                   G1Xyzz *__restrict__ out) {
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < n_out; t += (size_t)gridDim.x * blockDim.x) {
    G1Xyzz acc = in[t * chunk];
    for (int i = 1; i < chunk; i++) acc = xyzz_add_lazy(acc, in[t * chunk + i]);
    out[t] = acc;
  }
}

// out[r] = sum of parts[r*groups .. (r+1)*groups), one block per set
__global__ void __launch_bounds__(256) k_set_sum(const G1Xyzz *__restrict__ parts, size_t groups,
                                                 G1Xyzz *__restrict__ out) {
  __shared__ G1Xyzz lds[256];
  const size_t r = blockIdx.x;
  G1Xyzz acc = G1Xyzz::inf();
  for (size_t g = threadIdx.x; g < groups; g += blockDim.x) acc = xyzz_add_lazy(acc, parts[r * groups + g]);
  lds[threadIdx.x] = acc;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) lds[threadIdx.x] = xyzz_add_lazy(lds[threadIdx.x], lds[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) out[r] = xyzz_canon(lds[0]);  // the host reads canonical coordinates
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

// ---------------------------------------------------------------- fixed-base tables
__global__ void __launch_bounds__(256) k_affine_to_xyzz(const G1Affine *__restrict__ in, size_t n,
                                                        G1Xyzz *__restrict__ out) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = xyzz_from_affine(in[i]);
}

__global__ void __launch_bounds__(256) k_dbl_times(G1Xyzz *__restrict__ x, size_t n, int times) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    G1Xyzz p = x[i];
    for (int k = 0; k < times; k++) p = xyzz_dbl(p);
    x[i] = p;
  }
}

// the window a table for n points uses: the shared-layout optimum for full-width scalars
static int table_window(size_t n) {
  // no near-tie preference for the shared tables: at 2^20 + 1 points c = 19 (W = 14) was taken
  // over c = 20 (W = 13, 2 % cheaper in plan_cost) and the 2^20 MSM over it ran 2.42 vs 2.01 ms
  // (deeper buckets: 56 vs 26 entries each, k_bucket_fixup 0.28 vs 0.07 ms)
  return best_window(n, 254, 22, true, 0, 1.0);
}

FixedBase *fixed_base_build_dev(Ctx *c, const G1Affine *points, size_t n) {
  FixedBase *fb = new FixedBase();
  try {
    fb->n = n;
    fb->c = table_window(n);
    fb->W = windows_for(254, fb->c);
    G1Affine *T = (G1Affine *)fb->table.ensure(sizeof(G1Affine) * n * fb->W);
    TNS_HIP(hipMemcpyAsync(T, points, sizeof(G1Affine) * n, hipMemcpyDeviceToDevice, c->stream));
    const size_t slab = std::min(n, (size_t)1 << 22);
    DevBuf xb, pb;
    G1Xyzz *X = (G1Xyzz *)xb.ensure(sizeof(G1Xyzz) * slab);
    Fq *pre = (Fq *)pb.ensure(sizeof(Fq) * slab);
    for (size_t off = 0; off < n; off += slab) {
      const size_t m = std::min(slab, n - off);
      k_affine_to_xyzz<<<grid_for(m, 256), 256, 0, c->stream>>>(points + off, m, X);
      TNS_LAUNCH_CHECK();
      for (int j = 1; j < fb->W; j++) {
        k_dbl_times<<<grid_for(m, 256), 256, 0, c->stream>>>(X, m, fb->c);
        TNS_LAUNCH_CHECK();
        xyzz_to_affine_batch_dev(c, X, m, T + (size_t)j * n + off, pre);
      }
    }
    TNS_HIP(hipStreamSynchronize(c->stream));
  } catch (...) {
    delete fb;
    throw;
  }
  return fb;
}

// the window table if the device has room for it: on an allocation failure the MSMs over these
// points run without one (per-window buckets, same results) and nothing is cached
FixedBase *fixed_base_try_build(Ctx *c, const G1Affine *points, size_t n) {
  try {
    return fixed_base_build_dev(c, points, n);
  } catch (const Error &e) {
    if (e.code != TNS_ERR_OOM) throw;
    (void)hipGetLastError();  // clear the failed allocation's sticky status
    return nullptr;
  }
}

const FixedBase *srs_fixed_base(Ctx *c, const Srs &srs, size_t n) {
  if (n < ((size_t)1 << 16) || !c->msm_tables) return nullptr;
  if (srs.held < n) return nullptr;  // a shard's table covers its held points (tns_msm_sharded)
  if (!srs.fb) srs.fb = fixed_base_try_build(c, srs.points.as<G1Affine>(), srs.held);
  return srs.fb;
}

// ---------------------------------------------------------------- driver
// sum over each set of the sets x n array X (device) -> out (sets, device)
static void sum_sets(hipStream_t st, G1Xyzz *X, int sets, size_t n, G1Xyzz *tmp, G1Xyzz *out) {
  G1Xyzz *src = X, *dst = tmp;
  while (n > 128 && n % 8 == 0) {  // short chains: these passes are latency-bound
    const size_t n_out = (size_t)sets * (n / 8);
    k_sum_chunks<<<grid_for(n_out, 64, 1u << 30), 64, 0, st>>>(src, n_out, 8, dst);
    TNS_LAUNCH_CHECK();
    std::swap(src, dst);
    n /= 8;
  }
  k_set_sum<<<sets, 256, 0, st>>>(src, n, out);
  TNS_LAUNCH_CHECK();
}

// One MSM in flight on a lane: launched by msm_launch, completed by msm_complete.
struct MsmJob {
  MsmLane *lane = nullptr;
  bool immediate = false;  // result already known (n == 0, all scalars zero)
  G1Xyzz result;
  bool tiny = false;       // k_msm_tiny path: one point in the lane's pinned buffer
  MsmPlan P;
  int L0 = 0, nbits = 0, specs = 0;
  // between the sort phase and the accumulation phase
  bool sorted = false;
  bool sort_pending = false;        // bucket_sort_begin done, msm_finish_sort not yet
  bool passes_pending = false;      // bucket_sort_passes not yet queued
  BucketSortJob bs;
  hipEvent_t sorted_ev = nullptr;   // recorded on the lane once the bucket order exists
  std::unique_ptr<ProfScope> sort_prof;  // "msm_sort" timing from pass 1 to the last pass
  Ctx *ctx = nullptr;
  const G1Affine *points = nullptr;
  uint32_t *keys2 = nullptr, *vals2 = nullptr, *bstart = nullptr, *bend = nullptr, *valid = nullptr;
  int ks = 0, acc_k = 0;
  size_t nchunks = 0, n = 0;
  G1Xyzz *buckets = nullptr;  // set before the accumulation (a two-set tail: the pair's buckets adjoin)
  // where msm_complete finds the per-set sums: the slot of res_lane (this lane, or the lane that ran
  // a two-set tail), set res_set of res_sets
  MsmLane *res_lane = nullptr;
  int res_set = 0, res_sets = 1;
};

// ---------------------------------------------------------------- lane readbacks
struct PubArgs {
  const uint32_t *src[4];
  uint32_t words[4];
  int n;
};
constexpr size_t LANE_MAPPED_DATA[3] = {256, 512, 1024};  // slot data offsets; flags at 64 * slot
constexpr size_t LANE_MAPPED_BYTES = 1024 + 65536;

__global__ void __launch_bounds__(256) k_lane_publish(PubArgs a, uint32_t *dst, uint32_t *flag, uint32_t seq) {
  uint32_t off = 0;
  for (int k = 0; k < a.n; k++) {
    for (uint32_t i = threadIdx.x; i < a.words[k]; i += blockDim.x) dst[off + i] = a.src[k][i];
    off += a.words[k];
  }
  __threadfence_system();  // every thread's words reach host memory before the flag
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

void lane_publish(MsmLane &ln, int slot, int n, const void *const *src, const size_t *bytes) {
  char *m = (char *)ln.mapped.ensure(LANE_MAPPED_BYTES);
  (void)m;
  PubArgs a{};
  size_t total = 0;
  a.n = n;
  for (int k = 0; k < n; k++) {
    a.src[k] = (const uint32_t *)src[k];
    a.words[k] = (uint32_t)(bytes[k] / 4);
    total += bytes[k];
  }
  const size_t cap = (slot == 2 ? LANE_MAPPED_BYTES : LANE_MAPPED_DATA[slot + 1]) - LANE_MAPPED_DATA[slot];
  if (total > cap) throw Error(TNS_ERR_DEVICE, "lane readback larger than its slot");
  const uint32_t seq = ++ln.pub_seq;
  ln.slot_seq[slot] = seq;
  char *dev = (char *)ln.mapped.dev;
  k_lane_publish<<<1, 256, 0, ln.stream>>>(a, (uint32_t *)(dev + LANE_MAPPED_DATA[slot]), (uint32_t *)(dev + 64 * slot),
                                           seq);
  TNS_LAUNCH_CHECK();
}

void lane_publish_slot(MsmLane &ln, int slot, uint32_t **data, uint32_t **flag, uint32_t *seq) {
  ln.mapped.ensure(LANE_MAPPED_BYTES);
  *seq = ++ln.pub_seq;
  ln.slot_seq[slot] = *seq;
  char *dev = (char *)ln.mapped.dev;
  *data = (uint32_t *)(dev + LANE_MAPPED_DATA[slot]);
  *flag = (uint32_t *)(dev + 64 * slot);
}

// the slot's publish has landed (no wait)
static bool lane_ready(MsmLane &ln, int slot) {
  const uint32_t *flag = (const uint32_t *)((const char *)ln.mapped.p + 64 * slot);
  return __atomic_load_n(flag, __ATOMIC_ACQUIRE) == ln.slot_seq[slot];
}

const void *lane_wait(MsmLane &ln, int slot) {
  const char *m = (const char *)ln.mapped.p;
  const uint32_t *flag = (const uint32_t *)(m + 64 * slot), seq = ln.slot_seq[slot];
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned spin = 1; __atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq; spin++) {
    if ((spin & 4095) == 0) {  // a faulted stream reports here instead of leaving the flag unset
      const hipError_t e = hipStreamQuery(ln.stream);
      if (e != hipSuccess && e != hipErrorNotReady) TNS_HIP(e);
      if (e == hipSuccess && __atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq)
        throw Error(TNS_ERR_DEVICE, "lane readback: stream idle without its publish");
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > 120.0)
        throw Error(TNS_ERR_DEVICE, "lane readback did not arrive within 120 s");
    }
  }
  return m + LANE_MAPPED_DATA[slot];
}

// the largest bit length of Montgomery scalars; the sort then reads them as they are
// (SortInput::mont: canonicalised in its digit pass instead of through a canonical copy)
// With a plan hint for n scalars (the lane's previous MSM of Montgomery scalars: a proof's value
// commitment is the same shape every call) pass 1's count kernel computes the bit length too and
// the sort keeps its histograms when the bit length confirms the plan (else it recounts): one read
// of the scalars and one launch less (C4's value commitment: k_scalar_bits 0.26 ms + the count).
static SortInput bits_launch(MsmLane &ln, const Fr *scalars, size_t n) {
  unsigned *d_bits = (unsigned *)ln.ws[4].ensure(2 * sizeof(unsigned));  // (then the sort's two counters)
  TNS_HIP(hipMemsetAsync(d_bits, 0, sizeof(unsigned), ln.stream));
  SortInput in;
  in.fr = scalars;
  in.mont = true;
  const MsmLane::PlanHint &h = ln.hint;
  // (narrow per-window plans -- the trace values -- also get their canonical low 64 bits written)
  const bool narrow = !h.shared && h.c * h.W <= 64;
  if (!(h.n == n && h.c > 0 &&
        bucket_sort_precount_bits(ln, scalars, n, h.c, h.W, h.shared, h.bucket_bits, d_bits, in, narrow))) {
    k_scalar_bits<<<grid_for(n, 256, 2048), 256, 0, ln.stream>>>(scalars, n, d_bits, nullptr);
    TNS_LAUNCH_CHECK();
  }
  const void *src[1] = {d_bits};
  const size_t by[1] = {sizeof(unsigned)};
  lane_publish(ln, LANE_SLOT_BITS, 1, src, by);
  return in;
}

static unsigned bits_result(MsmLane &ln) { return *(const unsigned *)lane_wait(ln, LANE_SLOT_BITS); }

// Entries per accumulation thread.  Per-window plans (the narrow commitments: runs of a few
// entries, flush- and latency-bound): 128, halved down to 32 while the MSM gives fewer than
// ACC_THREADS_CU threads per CU -- short chunks shorten each thread's dependent chain.
// Table-window plans (full-width scalars) whose count the sort read back: the largest chunk
// <= 128 that fills whole rounds of the resident blocks (fewer chunks, fewer head/tail partials
// for the fixup: C2 2.17 -> 2.11 ms; the 2^24 openings keep 128, `profiles/r02_ab_acc_rounds.txt`).
constexpr int ACC_THREADS_CU = 1024;
static int acc_chunk(Ctx *ctx, size_t entries, bool table_plan) {
  if (!table_plan) {
    const size_t want = (size_t)ctx->num_cu * ACC_THREADS_CU;
    int k = 128;
    while (k > 32 && entries / k < want) k /= 2;
    return k;
  }
  static const int bpc = [] {  // resident blocks of 256 threads per CU (VGPR-bound: 3)
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_accumulate<false>, 256, 0) != hipSuccess || b < 1) b = 3;
    return b;
  }();
  const size_t slots = (size_t)ctx->num_cu * bpc * 256, kmax = 128;
  const size_t rounds = std::max<size_t>(1, (entries + kmax * slots - 1) / (kmax * slots));
  const size_t k = (entries + rounds * slots - 1) / (rounds * slots);
  return (int)std::max<size_t>(16, std::min<size_t>(kmax, k));
}

// Phase 1 on lane `ln` (asynchronous): plan, digits and the bucket order.  Trivial cases
// (all scalars zero, n <= 64) finish here.  `sorted` (optional) is recorded on the lane once
// the bucket order exists (or right away when there is none).
// canon: the canonical scalars from bits_launch (n > 64).
// defer: stop before the bucket sort's host wait (its last pass's readback); msm_finish_sort
// completes it, so a pair of MSMs can queue both lanes' passes before either waits.
static void msm_finish_sort(MsmJob &J);
static void msm_launch_sort(Ctx *ctx, MsmLane &ln, const G1Affine *points, const Fr *scalars, const SortInput &in,
                            size_t n, const FixedBase *fb, unsigned bits, MsmJob &J, hipEvent_t sorted = nullptr,
                            bool defer = false, size_t fb_off = 0) {
  J.lane = &ln;
  J.ctx = ctx;
  J.sorted_ev = sorted;
  hipStream_t st = ln.stream;
  auto record_now = [&]() {
    if (J.sorted_ev) TNS_HIP(hipEventRecord(J.sorted_ev, st));
    J.sorted_ev = nullptr;
  };
  if (n == 0 || bits == 0) {  // all scalars zero
    J.immediate = true;
    J.result = G1Xyzz::inf();
    record_now();
    return;
  }
  if (n <= 64) {
    G1Xyzz *d = (G1Xyzz *)ln.ws[0].ensure(sizeof(G1Xyzz));
    k_msm_tiny<<<1, 64, 0, st>>>(points, scalars, (int)n, d);
    TNS_LAUNCH_CHECK();
    const void *src[1] = {d};
    const size_t by[1] = {sizeof(G1Xyzz)};
    lane_publish(ln, LANE_SLOT_SUMS, 1, src, by);
    J.tiny = true;
    record_now();
    return;
  }
  if (n >= ((size_t)1 << 31)) throw Error(TNS_ERR_COMMITMENT, "MSM larger than 2^31 points");

  // plan: per-window layout, or the shared layout when a fixed-base table covers the points
  MsmPlan &P = J.P;
  P = MsmPlan();
  P.c = best_window(n, (int)bits, 20, false, 23);
  P.W = windows_for((int)bits, P.c);
  if (fb && ctx->msm_tables && fb->n >= fb_off + n && (uint64_t)fb->n * fb->W < ((uint64_t)1 << 31)) {
    const int Ws = windows_for((int)bits, fb->c);
    if (Ws <= fb->W && plan_cost(n, Ws, fb->c, 1) < plan_cost(n, P.W, P.c, P.W)) {
      P.shared = true;
      P.c = fb->c;
      P.W = Ws;
      P.stride = fb->n;
      points = fb->table.as<G1Affine>() + fb_off;  // T[w n + fb_off + i]: value w stride + i
    }
  }
  finish_plan(P);
  if (in.mont && in.fr && !in.u64) ln.hint = MsmLane::PlanHint{n, P.c, P.W, P.end_bit - 1, P.shared};
  SortInput in2 = in;
  if (in.low64 && bits <= 64) {  // the scalars fit 64 bits: the sort reads their canonical low words
    in2.u64 = in.low64;
    in2.n_u64 = n;
    in2.fr = nullptr;
    in2.mont = false;
  }
  const size_t total = (size_t)P.W * n;
  if (total >= ((size_t)1 << 31)) throw Error(TNS_ERR_COMMITMENT, "MSM too large for one sort");

  const int acc_k = acc_chunk(ctx, total, false);  // from the bound; table plans refine it from the sort's count
  J.points = points;
  J.acc_k = acc_k;
  J.nchunks = (total + acc_k - 1) / acc_k;
  J.n = n;
  J.sort_prof.reset(new ProfScope(ctx->prof, st, "msm_sort", 32.0 * n + 16.0 * total));
  J.valid = (uint32_t *)ln.ws[4].ensure(2 * sizeof(uint32_t));  // entries; [1]: a run crosses a chunk
  bucket_sort_begin(ln, in2, n, P.c, P.W, P.shared, (uint32_t)P.stride, P.end_bit - 1, J.valid, J.bs);
  J.sort_pending = true;
  J.passes_pending = true;
  if (!defer) msm_finish_sort(J);
}

// the bucket sort's passes after pass 1, up to the last pass's readback (no host wait)
static void msm_sort_passes(MsmJob &J) {
  if (!J.passes_pending) return;
  J.passes_pending = false;
  bucket_sort_passes(J.bs);
}

// the bucket sort's last stage (waits for its last-pass readback), then the sorted state
static void msm_finish_sort(MsmJob &J) {
  if (!J.sort_pending) return;
  msm_sort_passes(J);
  J.sort_pending = false;
  const BucketOrder o = bucket_sort_finish(J.bs);
  J.sort_prof.reset();  // the stage's end event, after the last pass on the lane
  if (o.entries != SIZE_MAX && J.P.shared) {  // table plans: chunks sized from the actual entry count
    J.acc_k = acc_chunk(J.ctx, o.entries, true);
    J.nchunks = std::max<size_t>(1, (o.entries + J.acc_k - 1) / J.acc_k);
  }
  J.keys2 = o.keys;
  J.vals2 = o.vals;
  J.bstart = o.bstart;
  J.bend = o.bstart + 1;
  J.ks = o.ks;
  J.sorted = true;
  if (J.sorted_ev) TNS_HIP(hipEventRecord(J.sorted_ev, J.lane->stream));
  J.sorted_ev = nullptr;
}

// Phase 2 (asynchronous): accumulation, bucket fixup, reduction and the per-set sums' readback.
// `accumulated` (optional) is recorded on the lane right after the accumulation kernel.
static void msm_launch_accumulate(Ctx *ctx, MsmJob &J, hipEvent_t accumulated, hipStream_t on = nullptr) {
  if (!J.sorted) {  // immediate / tiny: done in phase 1
    if (accumulated) TNS_HIP(hipEventRecord(accumulated, on ? on : J.lane->stream));
    return;
  }
  MsmLane &ln = *J.lane;
  hipStream_t st = on ? on : ln.stream;
  if (!J.buckets) J.buckets = (G1Xyzz *)ln.ws[5].ensure(sizeof(G1Xyzz) * J.P.nb);
  HeadTail *ht = (HeadTail *)ln.ws[6].ensure(sizeof(HeadTail) * J.nchunks);
  {
    TNS_PROF_ON(ctx, st, "msm_accumulate", 96.0 * J.n);  // 96 B per (scalar, point) pair
    uint2 *cbk = (uint2 *)ln.ws[16].ensure(sizeof(uint2) * J.nchunks);
    auto acc = J.keys2 ? k_accumulate<true> : k_accumulate<false>;
    acc<<<grid_for(J.nchunks, 256, 1u << 30), 256, 0, st>>>(J.keys2, J.vals2, J.valid, J.points, J.buckets, ht,
                                                            J.nchunks, J.ks, J.acc_k, J.bstart, J.P.nb, cbk,
                                                            J.valid + 1);
    TNS_LAUNCH_CHECK();
  }
  if (accumulated) TNS_HIP(hipEventRecord(accumulated, st));
}

// two sorted MSMs whose tails can run as one two-set launch sequence: the same bucket-set shape
static bool same_tail_shape(const MsmJob &a, const MsmJob &b) {
  return a.sorted && b.sorted && a.P.shared == b.P.shared && a.P.Wr == b.P.Wr && a.P.half == b.P.half;
}

// The accumulation's tail -- bucket fixup, reduction and the per-set sums' readback -- for nj = 1
// MSM, or nj = 2 of the same shape (same_tail_shape, buckets adjoining: J[1]->buckets ==
// J[0]->buckets + nb) as ONE sequence of launches on lane `run` whose grids cover both (a pair's two
// tails side by side on two lanes were short chains at low occupancy each, and the second lane's
// fixup took 0.97 ms against 0.38 ms for the same work on the first).
static void msm_launch_tails(Ctx *ctx, MsmJob *const *J, int nj, MsmLane &run) {
  for (int j = 0; j < nj; j++) {
    J[j]->res_lane = &run;
    J[j]->res_set = j;
    J[j]->res_sets = nj;
  }
  if (!J[0]->sorted) return;
  hipStream_t st = run.stream;
  const MsmPlan &P = J[0]->P;
  if (nj == 2 && (!same_tail_shape(*J[0], *J[1]) || J[1]->buckets != J[0]->buckets + P.nb))
    throw Error(TNS_ERR_DEVICE, "two-set MSM tail over MSMs of different shapes");
  {
    TNS_PROF_ON(ctx, st, "msm_fixup", 0.0);
    FixupArgs FA{};
    int max_levels = 0;
    size_t max_nb = 0;
    for (int j = 0; j < nj; j++) {
      MsmJob &X = *J[j];
      FixLevels &F = FA.s[j].F;
      size_t groups = X.nchunks / FIX_FAN, off = 0;
      while (F.n < FIX_LEVELS && groups >= 2) {  // level sizes: nchunks/F, /F^2, ...
        F.len[F.n + 1] = groups;
        off += groups;
        groups /= FIX_FAN;
        F.n++;
      }
      if (F.n) {
        G1Xyzz *base = (G1Xyzz *)X.lane->fix.ensure(sizeof(G1Xyzz) * off);
        size_t o = 0;
        for (int l = 1; l <= F.n; o += F.len[l], l++) F.lv[l] = base + o;
      }
      max_levels = std::max(max_levels, F.n);
      FA.s[j] = FixupSet{X.bstart, X.bend, X.valid, (const HeadTail *)X.lane->ws[6].p, F, X.buckets, X.P.nb, X.acc_k};
      max_nb = std::max(max_nb, X.P.nb);
    }
    for (int l = 1; l <= max_levels; l++) {
      FixLevelArgs LA{};
      size_t max_groups = 0;
      for (int j = 0; j < nj; j++) {
        const FixLevels &F = FA.s[j].F;
        const MsmJob &X = *J[j];
        LA.s[j] = FixLevelSet{X.valid, FA.s[j].ht, F.lv[l - 1], F.lv[l], (const uint2 *)X.lane->ws[16].p,
                              l <= F.n ? F.len[l] : 0, X.acc_k};
        if (l <= F.n) max_groups = std::max(max_groups, F.len[l]);
      }
      k_fix_level<<<dim3(grid_for(max_groups * FIX_FAN, 256, 1u << 30), nj), 256, 0, st>>>(LA, l);
      TNS_LAUNCH_CHECK();
    }
    k_bucket_fixup<<<dim3(grid_for(max_nb, 256), nj), 256, 0, st>>>(FA);
    TNS_LAUNCH_CHECK();
  }
  // bucket reduction (see the header): running sums over groups of L0 buckets, then
  // the weighted group sum  sum_g g S_g = sum_b 2^b M_b,  M_b = sum_{g: bit b of g} S_g,
  // as nbits + 2 plain sums (the M_b and sum_g T_g in two halves) -- short dependency chains only.
  // Up to 2^19 buckets per set the chains are the latency: groups of 4 and masked-sum chunks of 8
  // (C2, 2^20 points: 2.73 -> 2.65 ms); from 2^21 buckets groups of 16 stay the fastest (2^22,
  // 2^24; 8: +0.19 ms, 32: +0.63 ms per C4 step, r05 A/B).  c >= 4: half >= 8, so g >= 2.
  const int sets = P.Wr * nj;
  const bool small_sets = P.half <= ((size_t)1 << 19);
  int L0 = (int)std::min<size_t>(small_sets ? 4 : RED_L, P.half / 2);
  const size_t g1 = P.half / L0;
  // a second level (k_reduce_level2, groups of L1 = 4) when the first leaves many groups
  int L1 = g1 >= ((size_t)1 << 13) ? 4 : 0;
  if (L1 && g1 / L1 < 2) L1 = 0;
  const size_t g = L1 ? g1 / L1 : g1;
  int nbits = 0;
  while (((size_t)1 << nbits) < g) nbits++;
  const int specs = nbits + 2;
  {
    TNS_PROF_ON(ctx, st, "msm_reduce", 128.0 * P.nb * nj);
    G1Xyzz *T = (G1Xyzz *)run.ws[7].ensure(sizeof(G1Xyzz) * 2 * sets * (g1 + (L1 ? g : 0)));
    G1Xyzz *S = T + (size_t)sets * g1;
    k_reduce_level<<<grid_for((size_t)sets * g1, 64, 1u << 30), 64, 0, st>>>(J[0]->buckets, sets, P.half, L0, T, S);
    TNS_LAUNCH_CHECK();
    if (L1) {
      G1Xyzz *V = S + (size_t)sets * g1, *S2 = V + (size_t)sets * g;
      int lg0 = 0;
      while ((1 << lg0) < L0) lg0++;
      k_reduce_level2<<<grid_for((size_t)sets * g, 64, 1u << 30), 64, 0, st>>>(T, S, sets, g1, L1, lg0, V, S2);
      TNS_LAUNCH_CHECK();
      T = V;
      S = S2;
      L0 *= L1;  // the masked sums' weight (msm_complete's doublings)
    }
    const int CH = (int)std::min<size_t>(small_sets || L1 ? 8 : 16, g / 2);
    const size_t nch = g / (2 * (size_t)CH);
    const size_t nparts = (size_t)sets * specs * nch;
    G1Xyzz *parts = (G1Xyzz *)run.ws[8].ensure(sizeof(G1Xyzz) * (2 * nparts + (size_t)sets * specs));
    G1Xyzz *tmp = parts + nparts, *out = tmp + nparts;
    const bool tree = nch % 64 == 0;  // each wave adds its 64 chunk sums by a butterfly
    k_masked_sums<<<grid_for(nparts, 64, 1u << 30), 64, 0, st>>>(T, S, sets, g, nbits, CH, parts, tree);
    TNS_LAUNCH_CHECK();
    sum_sets(st, parts, sets * specs, tree ? nch / 64 : nch, tmp, out);
    // the per-set sums, then each MSM's number of sorted non-zero digits (= mixed additions of
    // k_accumulate, profiling)
    const void *src[3] = {out, J[0]->valid, nj == 2 ? J[1]->valid : nullptr};
    const size_t by[3] = {sizeof(G1Xyzz) * sets * specs, sizeof(uint32_t), sizeof(uint32_t)};
    lane_publish(run, LANE_SLOT_SUMS, 1 + nj, src, by);
  }
  for (int j = 0; j < nj; j++) {
    J[j]->L0 = L0;
    J[j]->nbits = nbits;
    J[j]->specs = specs;
  }
}

static void msm_launch_reduce(Ctx *ctx, MsmJob &J, hipEvent_t accumulated = nullptr) {
  msm_launch_accumulate(ctx, J, accumulated);
  MsmJob *one[1] = {&J};
  msm_launch_tails(ctx, one, 1, *J.lane);
}

// Wait for the tail's readback and finish on the host: R = sum_g T_g + L0 * sum_b 2^b M_b per
// set, then Horner over the windows (per-window layout).
static G1Xyzz msm_complete(Ctx *ctx, MsmJob &J) {
  if (J.immediate) return J.result;
  const void *hp = lane_wait(J.res_lane ? *J.res_lane : *J.lane, LANE_SLOT_SUMS);
  if (J.tiny) return *(const G1Xyzz *)hp;
  const MsmPlan &P = J.P;
  const G1Xyzz *all = (const G1Xyzz *)hp;
  const G1Xyzz *fin = all + (size_t)J.res_set * P.Wr * J.specs;
  const uint32_t *cnt = (const uint32_t *)(all + (size_t)J.res_sets * P.Wr * J.specs);
  ctx->prof.add_ops("msm_accumulate", (double)cnt[J.res_set]);
  std::vector<G1Xyzz> Rw(P.Wr);
  for (int r = 0; r < P.Wr; r++) {
    const G1Xyzz *f = &fin[(size_t)r * J.specs];
    G1Xyzz acc = G1Xyzz::inf();
    for (int b = J.nbits - 1; b >= 0; b--) acc = xyzz_add(xyzz_dbl(acc), f[b]);
    for (int L = J.L0; L > 1; L >>= 1) acc = xyzz_dbl(acc);
    Rw[r] = xyzz_add(xyzz_add(f[J.nbits], f[J.nbits + 1]), acc);
  }
  if (P.shared) return Rw[0];
  G1Xyzz acc = Rw[P.W - 1];
  for (int w = P.W - 2; w >= 0; w--) {
    for (int k = 0; k < P.c; k++) acc = xyzz_dbl(acc);
    acc = xyzz_add(acc, Rw[w]);
  }
  return acc;
}

G1Xyzz msm_dev(Ctx *ctx, const G1Affine *points, const Fr *scalars, size_t n, const FixedBase *fb, size_t fb_off) {
  if (n == 0) return G1Xyzz::inf();
  MsmLane &ln = ctx->lanes[0];
  unsigned bits = 254;
  SortInput in;
  if (n > 64) {
    in = bits_launch(ln, scalars, n);
    bits = bits_result(ln);
  }
  MsmJob J;
  msm_launch_sort(ctx, ln, points, scalars, in, n, fb, bits, J, nullptr, false, fb_off);
  msm_launch_reduce(ctx, J);
  return msm_complete(ctx, J);
}

void msm_pair_dev(Ctx *ctx, const MsmArgs &a, const MsmArgs &b, G1Xyzz out[2]) {
  if (a.late && !b.late) {  // the late vector goes second (lane 1)
    G1Xyzz o[2];
    msm_pair_dev(ctx, b, a, o);
    out[0] = o[1];
    out[1] = o[0];
    return;
  }
  MsmLane &l0 = ctx->lanes[0], &l1 = ctx->lanes[1];
  // lane 1 starts after everything already queued on the context stream (its inputs)
  hipEvent_t ready;
  TNS_HIP(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
  TNS_HIP(hipEventRecord(ready, ctx->stream));
  TNS_HIP(hipStreamWaitEvent(l1.stream, ready, 0));
  (void)hipEventDestroy(ready);
  unsigned ba = 254, bb = 254;
  SortInput ca, cb;
  // canonical inputs (the opening quotients) and raw u64 inputs (trace addresses, lookup
  // indices) come with their bit lengths on the device
  auto start = [&](MsmLane &ln, const MsmArgs &x) -> SortInput {
    if (x.prep) x.prep(ln.stream);
    if (x.n <= 64) return SortInput();
    if (!x.canon_bits) return bits_launch(ln, x.scalars, x.n);
    if (x.plan_bits <= 0) {  // (plan_bits: nothing to read back)
      const void *src[1] = {x.canon_bits};
      const size_t by[1] = {sizeof(unsigned)};
      lane_publish(ln, LANE_SLOT_BITS, 1, src, by);
    }
    SortInput in;
    if (x.u64) {
      in.u64 = x.u64;
      in.n_u64 = x.n_u64;
    } else {
      in.fr = x.canon ? x.canon : x.scalars;
      in.precounted = x.precounted;
      in.pre_c = x.pre_c;
      in.pre_W = x.pre_W;
    }
    return in;
  };
  MsmJob ja, jb;
  if (b.late) {
    // b's scalars are still being uploaded (HostUpload, a helper thread): a's MSM is queued whole
    // first -- sort, accumulation, tail -- so it runs under the upload; b's prep then waits for
    // the upload and b's MSM follows on lane 1
    ca = start(l0, a);
    if (a.n > 64) ba = bits_result(l0);
    msm_launch_sort(ctx, l0, a.points, a.scalars, ca, a.n, a.fb, ba, ja);
    msm_launch_reduce(ctx, ja);
    if (b.chunks > 1) {  // one MSM per uploaded chunk, each as soon as it lands
      if ((int)b.chunk_off.size() != b.chunks + 1 || b.chunk_off.back() != b.n)
        throw Error(TNS_ERR_INVALID_PARAMETERS, "chunk offsets do not cover the scalars");
      G1Xyzz acc = G1Xyzz::inf();
      for (int k = 0; k < b.chunks; k++) {
        const size_t off = b.chunk_off[k], cnt = b.chunk_off[k + 1] - off;
        if (!cnt) continue;
        MsmArgs bk{b.points + off, b.scalars + off, cnt, b.fb};
        bk.prep = [&b, k](hipStream_t s) { b.chunk_prep(k, s); };
        MsmJob jk;
        unsigned bk_bits = 254;
        const SortInput ck = start(l1, bk);
        if (cnt > 64) bk_bits = bits_result(l1);
        msm_launch_sort(ctx, l1, bk.points, bk.scalars, ck, cnt, b.fb, bk_bits, jk, nullptr, false, off);
        msm_launch_reduce(ctx, jk);
        acc = xyzz_add(acc, msm_complete(ctx, jk));  // the lane's host buffer serves the next chunk
      }
      out[0] = msm_complete(ctx, ja);
      out[1] = acc;
      return;
    }
    cb = start(l1, b);
    if (b.n > 64) bb = bits_result(l1);
    msm_launch_sort(ctx, l1, b.points, b.scalars, cb, b.n, b.fb, bb, jb);
    msm_launch_reduce(ctx, jb);
    out[0] = msm_complete(ctx, ja);
    out[1] = msm_complete(ctx, jb);
    return;
  }
  ca = start(l0, a);
  cb = start(l1, b);
  if (a.n > 64) ba = a.plan_bits > 0 ? (unsigned)a.plan_bits : bits_result(l0);
  if (b.n > 64) bb = b.plan_bits > 0 ? (unsigned)b.plan_bits : bits_result(l1);
  hipEvent_t sa = nullptr, sb = nullptr;
  TNS_HIP(hipEventCreateWithFlags(&sa, hipEventDisableTiming));
  TNS_HIP(hipEventCreateWithFlags(&sb, hipEventDisableTiming));
  // both lanes' passes are queued before either lane's host wait (the last pass's readback), and
  // each lane's last pass follows its own readback: the two sorts run side by side and neither
  // waits for the other's first passes (profiles/r02_ab_sort_overlap.txt, r05_ab_sort_overlap.txt)
  msm_launch_sort(ctx, l0, a.points, a.scalars, ca, a.n, a.fb, ba, ja, sa, true);
  msm_sort_passes(ja);
  msm_launch_sort(ctx, l1, b.points, b.scalars, cb, b.n, b.fb, bb, jb, sb, true);
  msm_sort_passes(jb);
  // Both accumulations go on the context's side stream (free here: its folds run before the
  // openings' MSMs), one after the other (each is VALU-bound on the whole chip: run together they
  // take as long), each as soon as its own sort is done: the first runs beside the rest of lane 1's
  // sort, which then finishes in the first accumulation's tail-off.  Waiting for both sorts first
  // left the chip to lane 1's last passes alone for ~1.2 ms; this is 0.4 ms faster per C4 step
  // (profiles/r06_ab_acc_stream.txt) -- lane 1's sort stage then spans the first accumulation.
  // A pair of table-window MSMs (the openings: full-width scalars, ~16 ms accumulations) runs both
  // tails after the second accumulation as ONE two-set launch sequence on lane 0 (tails under the
  // second accumulation took wave slots from it, profiles/r02_ab_tails_last.txt); the commitments
  // keep lane 0's tail under lane 1's accumulation (the 22-bit address MSM's 2^22-bucket reduction
  // is longer than the value accumulation).
  hipStream_t as = ctx->acc;
  msm_finish_sort(ja);
  hipEvent_t acc_a, acc_b;
  TNS_HIP(hipEventCreateWithFlags(&acc_a, hipEventDisableTiming));
  TNS_HIP(hipEventCreateWithFlags(&acc_b, hipEventDisableTiming));
  // a two-set tail needs the pair's buckets adjoining: room for both before acc a writes the first
  if (ja.sorted && ja.P.shared) ja.buckets = (G1Xyzz *)l0.ws[5].ensure(sizeof(G1Xyzz) * 2 * ja.P.nb);
  TNS_HIP(hipStreamWaitEvent(as, sa, 0));
  msm_launch_accumulate(ctx, ja, acc_a, as);
  msm_finish_sort(jb);
  const bool tails_last = ja.sorted && jb.sorted && ja.P.shared && jb.P.shared;
  const bool two_set = tails_last && same_tail_shape(ja, jb);
  if (two_set) jb.buckets = ja.buckets + ja.P.nb;
  TNS_HIP(hipStreamWaitEvent(as, sb, 0));
  msm_launch_accumulate(ctx, jb, acc_b, as);
  (void)hipEventDestroy(sa);
  (void)hipEventDestroy(sb);
  TNS_HIP(hipStreamWaitEvent(l0.stream, tails_last ? acc_b : acc_a, 0));
  if (two_set) {
    MsmJob *both[2] = {&ja, &jb};
    msm_launch_tails(ctx, both, 2, l0);
  } else {
    TNS_HIP(hipStreamWaitEvent(l1.stream, acc_b, 0));
    MsmJob *one_a[1] = {&ja}, *one_b[1] = {&jb};
    msm_launch_tails(ctx, one_a, 1, l0);
    msm_launch_tails(ctx, one_b, 1, l1);
  }
  (void)hipEventDestroy(acc_a);
  (void)hipEventDestroy(acc_b);
  // two tails on two lanes: the host's part (bucket-sum Horner, ~20-45 us) of whichever lands
  // first runs while the other lane's tail still runs on the device
  if (!two_set && jb.res_lane && jb.res_lane != ja.res_lane && jb.sorted && ja.sorted) {
    // (bounded: past it the plain order below, whose waits report a faulted stream)
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned spin = 1; !lane_ready(*ja.res_lane, LANE_SLOT_SUMS) && !lane_ready(*jb.res_lane, LANE_SLOT_SUMS);
         spin++)
      if ((spin & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(500)) break;
    if (!lane_ready(*ja.res_lane, LANE_SLOT_SUMS) && lane_ready(*jb.res_lane, LANE_SLOT_SUMS)) {
      out[1] = msm_complete(ctx, jb);
      out[0] = msm_complete(ctx, ja);
      return;
    }
  }
  out[0] = msm_complete(ctx, ja);
  out[1] = msm_complete(ctx, jb);
}

}  // namespace tns
