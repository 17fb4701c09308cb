// mle.hip -- multilinear-extension fold/evaluate and the fused sum-check round kernel.
//
// Reference semantics: MultilinearExtension::evaluate / partial_evaluate
// (src/polynomials.rs:85-161) with variable j <-> index bit j (LSB first), and
// SumCheck::prove (src/sumcheck.rs:56-110), whose round r sums the closure at
// (r_0..r_{r-1}, X, suffix bits) for X in {0,1,2,3}.
//
// Instead of the reference's O(N * n) evaluate per hypercube point we keep each
// MLE as a table and bind one variable per round:  T'[s] = T[2s] + r (T[2s+1] - T[2s]).
// The round-k values at X are T_k[2s] + X (T_k[2s+1] - T_k[2s]).  One launch fuses
// the fold by r_{k-1} with the round-k sums, so every round streams each table
// once: read 32 B x (4 entries), write 32 B x 2 per output pair -- 48 B per input
// entry, 96 B per entry over the whole chain (HBM-bound).
#include <hip/hip_runtime.h>

#include <cstring>

#include "common.hpp"
#include "hostfield.hpp"

namespace tns {

constexpr int MAX_SC_TABLES = 4;
#ifndef TNS_SC_WAVES3
#define TNS_SC_WAVES3 3  // waves per SIMD asked of the round kernel for <= 3 tables (4: same time, spills)
#endif

struct ScTables {
  const Fr *in[MAX_SC_TABLES];
  Fr *out[MAX_SC_TABLES];
};
// ---------------------------------------------------------------- generic compositions
// A degree <= 3 composition sum_t c_t prod_{j in t} T_j over K <= 4 tables is rewritten on the
// host (sc_poly) in nested form
//     f = c + sum_i T_i (c_i + sum_{j >= i} T_j (c_ij + sum_{l >= j} c_ijl T_l))
// with the tables renumbered for the fewest products per point: the Twist-shaped
// A V - O O V + 2 O becomes V (A - O O) + 2 O, 2 products instead of 3.  The round kernel unrolls
// i, j, l at compile time (table values stay in registers, no run-time selects) and branches only
// on the uniform coefficient kinds; a coefficient multiplies only when it is not 1, -1 or 2.
constexpr int SC_SLOTS = 35;  // 1 constant + 4 linear + 10 quadratic + 20 cubic monomials
enum : int32_t { CK_ZERO = 0, CK_ONE = 1, CK_MONE = 2, CK_TWO = 3, CK_ANY = 4 };
// (the flags are 32-bit words: the kernel reads them with scalar loads.  As bytes they were
// global_load_ubyte -- gfx950 has no sub-dword scalar load -- each followed by a vmcnt(0) wait
// that also waited out the wave's table loads and fold stores: ~20 memory round trips per point)
struct ScPoly {
  Fr coef[SC_SLOTS];
  int32_t kind[SC_SLOTS];
  int32_t has_i[MAX_SC_TABLES];                  // some monomial starts with table i
  int32_t i_lin[MAX_SC_TABLES];                  // ... and i's inner part is more than c_i
  int32_t has_ij[MAX_SC_TABLES][MAX_SC_TABLES];  // some monomial starts with (i, j)
  int32_t ij_lin[MAX_SC_TABLES][MAX_SC_TABLES];  // ... and (i, j)'s inner part is more than c_ij
  int32_t ij_sq[MAX_SC_TABLES][MAX_SC_TABLES];   // ... and that inner part is c_ijj T_j alone: a square
};
__host__ __device__ constexpr int sc_slot1(int i) { return 1 + i; }
__host__ __device__ constexpr int sc_slot2(int i, int j) { return 5 + 4 * i - i * (i - 1) / 2 + (j - i); }
__host__ __device__ constexpr int sc_slot3(int i, int j, int l) {
  int s = 15;
  for (int a = 0; a < 4; a++)
    for (int b = a; b < 4; b++)
      for (int c = b; c < 4; c++) {
        if (a == i && b == j && c == l) return s;
        s++;
      }
  return -1;
}

// The nested form of a composition for one table order perm (perm[m] = the caller's table that
// kernel table m reads); returns its products per evaluation point.
static int sc_poly_for(const SumcheckTerm *terms, int n_terms, int k, const int *perm, ScPoly *out) {
  int inv[MAX_SC_TABLES] = {0, 0, 0, 0};
  for (int m = 0; m < k; m++) inv[perm[m]] = m;
  Fr acc[SC_SLOTS];
  bool used[SC_SLOTS] = {};
  for (int t = 0; t < SC_SLOTS; t++) acc[t] = Fr::zero();
  for (int t = 0; t < n_terms; t++) {
    int ix[3], d = 0;
    for (int j = 0; j < 3; j++)
      if (terms[t].tab[j] >= 0) ix[d++] = inv[terms[t].tab[j]];
    std::sort(ix, ix + d);
    const int slot = d == 0 ? 0 : d == 1 ? sc_slot1(ix[0]) : d == 2 ? sc_slot2(ix[0], ix[1]) : sc_slot3(ix[0], ix[1], ix[2]);
    acc[slot] = add(acc[slot], terms[t].coeff);
    used[slot] = true;
  }
  ScPoly q{};
  const Fr one = Fr::one(), two = add(one, one), mone = neg(one);
  int muls = 0;
  for (int t = 0; t < SC_SLOTS; t++) {
    q.coef[t] = acc[t];
    q.kind[t] = !used[t] || acc[t] == Fr::zero() ? CK_ZERO
                : acc[t] == one                 ? CK_ONE
                : acc[t] == mone                ? CK_MONE
                : acc[t] == two                 ? CK_TWO
                                                : CK_ANY;
  }
  for (int i = 0; i < k; i++) {
    for (int j = i; j < k; j++) {
      bool lin = false;
      for (int l = j; l < k; l++)
        if (q.kind[sc_slot3(i, j, l)]) {
          lin = true;
          muls += q.kind[sc_slot3(i, j, l)] == CK_ANY;
        }
      q.ij_lin[i][j] = lin;
      q.has_ij[i][j] = lin || q.kind[sc_slot2(i, j)];
      bool only_jj = lin && !q.kind[sc_slot2(i, j)];
      for (int l = j + 1; l < k; l++) only_jj = only_jj && !q.kind[sc_slot3(i, j, l)];
      q.ij_sq[i][j] = only_jj;  // T_j (c_ijj T_j) = c_ijj T_j^2
      if (lin) muls += 1;  // T_j * (c_ij + ...)
      else if (q.kind[sc_slot2(i, j)] == CK_ANY) muls += 1;
      q.i_lin[i] |= q.has_ij[i][j];
    }
    q.has_i[i] = q.i_lin[i] || q.kind[sc_slot1(i)];
    if (q.i_lin[i]) muls += 1;  // T_i * (c_i + ...)
    else if (q.kind[sc_slot1(i)] == CK_ANY) muls += 1;
  }
  if (out) *out = q;
  return muls;
}

// The table order with the fewest products (ties: the caller's order), and its nested form.
static ScPoly sc_poly(const SumcheckTerm *terms, int n_terms, int k, int perm[MAX_SC_TABLES]) {
  if (n_terms > 64) throw Error(TNS_ERR_INVALID_PARAMETERS, "at most 64 sum-check terms");
  for (int t = 0; t < n_terms; t++)
    for (int j = 0; j < 3; j++)
      if (terms[t].tab[j] >= k) throw Error(TNS_ERR_INVALID_PARAMETERS, "term references a missing table");
  int p[MAX_SC_TABLES] = {0, 1, 2, 3};
  int best = -1;
  do {
    const int m = sc_poly_for(terms, n_terms, k, p, nullptr);
    if (best < 0 || m < best) {
      best = m;
      std::copy(p, p + MAX_SC_TABLES, perm);
    }
  } while (std::next_permutation(p, p + k));
  ScPoly q;
  sc_poly_for(terms, n_terms, k, perm, &q);
  return q;
}

// ---------------------------------------------------------------- wave/block reductions
__device__ __forceinline__ Fr shfl_down_fr(const Fr &a, int d) {
  Fr r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = __shfl_down(a.v[i], d, 64);
  return r;
}

// Sum NV field elements across the block; thread 0 gets the result.  blockDim <= 1024.
template <int NV>
__device__ void block_sum_fr(Fr (&v)[NV], Fr *lds /* [NV][16] */) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
#pragma unroll
    for (int k = 0; k < NV; k++) {
      Fr o = shfl_down_fr(v[k], d);
      if (lane + d < 64) v[k] = add(v[k], o);
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < NV; k++) lds[k * 16 + wid] = v[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 0; k < NV; k++) {
      Fr s = lds[k * 16];
      for (int w = 1; w < nw; w++) s = add(s, lds[k * 16 + w]);
      v[k] = s;
    }
  }
}

// ---------------------------------------------------------------- fold
__global__ void __launch_bounds__(256) k_mle_fold(const Fr *__restrict__ in, Fr *__restrict__ out,
                                                  size_t half, Fr r) {
  for (size_t s = blockIdx.x * (size_t)blockDim.x + threadIdx.x; s < half;
       s += (size_t)gridDim.x * blockDim.x) {
    Fr a = in[2 * s], b = in[2 * s + 1];
    out[s] = add(a, mul(r, sub(b, a)));
  }
}

void mle_fold_dev(Ctx *c, const Fr *in, Fr *out, size_t half, const Fr &r) {
  k_mle_fold<<<grid_for(half, 256), 256, 0, c->stream>>>(in, out, half, r);
  TNS_LAUNCH_CHECK();
}

// Evaluate by nv successive folds (ping-pong in scratch).  point_host: nv Fr.
Fr mle_evaluate_dev(Ctx *c, const Fr *evals, unsigned nv, const Fr *point_host) {
  if (nv == 0) {
    Fr r;
    TNS_HIP(hipMemcpyAsync(&r, evals, sizeof(Fr), hipMemcpyDeviceToHost, c->stream));
    TNS_HIP(hipStreamSynchronize(c->stream));
    return r;
  }
  size_t n = (size_t)1 << nv;
  Fr *a = (Fr *)c->scratch[0].ensure(sizeof(Fr) * (n / 2));
  Fr *b = (Fr *)c->scratch[1].ensure(sizeof(Fr) * (n / 4 > 0 ? n / 4 : 1));
  const Fr *src = evals;
  Fr *dst = a;
  for (unsigned j = 0; j < nv; j++) {
    size_t half = n >> (j + 1);
    mle_fold_dev(c, src, dst, half, point_host[j]);
    src = dst;
    dst = (dst == a) ? b : a;
  }
  Fr r;
  TNS_HIP(hipMemcpyAsync(&r, src, sizeof(Fr), hipMemcpyDeviceToHost, c->stream));
  TNS_HIP(hipStreamSynchronize(c->stream));
  return r;
}

// ---------------------------------------------------------------- fused sum-check round
// A fold by r: T'[s] = T[2s] + r (T[2s+1] - T[2s]) for 2P outputs (the closure-free chain's
// single-round passes; 2P entries written, 4P read).
__global__ void __launch_bounds__(256) k_sc_fold(ScTables t, int k, size_t P, Fr r) {
  for (size_t s = blockIdx.x * (size_t)blockDim.x + threadIdx.x; s < P; s += (size_t)gridDim.x * blockDim.x) {
#pragma unroll
    for (int i = 0; i < MAX_SC_TABLES; i++) {
      if (i < k) {
        const Fr *p = t.in[i] + 4 * s;
        const Fr x0 = p[0], x1 = p[1], x2 = p[2], x3 = p[3];
        t.out[i][2 * s] = add(x0, mul(r, sub(x1, x0)));
        t.out[i][2 * s + 1] = add(x2, mul(r, sub(x3, x2)));
      }
    }
  }
}

// The round kernel's arithmetic runs in the lazy domain [0, 2M] of the MSM accumulation
// (bn254.hpp): products skip the final conditional subtraction (inputs <= 2M give results < 2M,
// 4M < 2^256), sums and differences reduce against 2M; values are canonicalised only where they
// leave the kernel (the round sums, the final table values).
__device__ __forceinline__ Fr sc_canon(Fr a) {
  reduce_once(a);  // [0, 2M] -> [0, M]
  reduce_once(a);  // M -> 0
  return a;
}
__device__ __forceinline__ Fr sc_mul(const Fr &a, const Fr &b) { return mul_lazy_dev(a, b); }
__device__ __forceinline__ Fr sc_sqr(const Fr &a) { return sqr_lazy_dev(a); }
__device__ __forceinline__ Fr sc_cmul(int32_t kind, const Fr &c, const Fr &v) {
  if (kind == CK_ONE) return v;
  if (kind == CK_MONE) return const_minus_dev<FrCfg, true>(v);  // 2M - v
  if (kind == CK_TWO) return add2_dev(v, v);
  return sc_mul(c, v);
}

// the composition at one point (table values v[0..K)), nested form of ScPoly; i, j, l are
// template parameters so every table value and coefficient slot is a compile-time index
template <int K, int I, int J, int L>
__device__ __forceinline__ void sc_eval_l(const ScPoly &q, const Fr (&v)[K], Fr &in2) {
  if constexpr (L < K) {
    constexpr int s3 = sc_slot3(I, J, L);
    if (q.kind[s3]) in2 = add2_dev(in2, sc_cmul(q.kind[s3], q.coef[s3], v[L]));
    sc_eval_l<K, I, J, L + 1>(q, v, in2);
  }
}
template <int K, int I, int J>
__device__ __forceinline__ void sc_eval_j(const ScPoly &q, const Fr (&v)[K], Fr &inner) {
  if constexpr (J < K) {
    if (q.has_ij[I][J]) {
      constexpr int s2 = sc_slot2(I, J);
      if (!q.ij_lin[I][J]) {
        inner = add2_dev(inner, sc_cmul(q.kind[s2], q.coef[s2], v[J]));
      } else if (q.ij_sq[I][J]) {  // c T_j^2: the dedicated square
              constexpr int s3 = sc_slot3(I, J, J);
        inner = add2_dev(inner, sc_cmul(q.kind[s3], q.coef[s3], sc_sqr(v[J])));
      } else {
              Fr in2 = q.coef[s2];
        sc_eval_l<K, I, J, J>(q, v, in2);
        inner = add2_dev(inner, sc_mul(v[J], in2));
      }
    }
    sc_eval_j<K, I, J + 1>(q, v, inner);
  }
}
template <int K, int I>
__device__ __forceinline__ void sc_eval_i(const ScPoly &q, const Fr (&v)[K], Fr &acc) {
  if constexpr (I < K) {
    if (q.has_i[I]) {
      constexpr int s1 = sc_slot1(I);
      if (!q.i_lin[I]) {
        acc = add2_dev(acc, sc_cmul(q.kind[s1], q.coef[s1], v[I]));
      } else {
              Fr inner = q.coef[s1];
        sc_eval_j<K, I, I>(q, v, inner);
        acc = add2_dev(acc, sc_mul(v[I], inner));
      }
    }
    sc_eval_i<K, I + 1>(q, v, acc);
  }
}
template <int K>
__device__ __forceinline__ Fr sc_eval(const ScPoly &q, const Fr (&v)[K]) {
  Fr acc = q.coef[0];  // the constant (zero when absent)
  sc_eval_i<K, 0>(q, v, acc);
  return acc;
}

// Where a round kernel's last workgroup leaves the round's four sums (fine-grained host memory,
// polled by the host: no stream synchronize, no second launch).
struct ScResult {
  Fr sums[4];
  uint32_t flag;
  // set by a device waiter whose 5 s bound for the host's challenge expired (it then released the
  // kernels behind it without sums): sc_wait reports that cause at once instead of a missing publish
  uint32_t wait_expired;
  uint32_t pad[6];
};

// A round's challenge handed to round kernels queued before it existed: the host writes r and then
// the flag into ScChal (fine-grained host memory); k_sc_wait_r, queued ahead of the round kernel,
// polls the flag and copies r into device memory (ScRDev) for the kernels behind it.  SC_CANCEL
// (host error path) or a 5 s bound sets `abort` instead, and the kernels behind it return at once.
struct ScChal {
  Fr r;
  uint32_t flag;
  uint32_t pad[7];
};
struct ScRDev {
  Fr r;
  uint32_t abort;
  uint32_t pad[7];
};
constexpr uint32_t SC_CANCEL = 0xFFFFFFFFu;

__global__ void __launch_bounds__(64) k_sc_wait_r(ScChal *chal, uint32_t seq, ScRDev *rd, ScResult *res) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
  uint32_t f;
  // (relaxed polls, one acquire fence after: an acquire load per poll invalidates the caches each
  // time -- measured 2-8x slower sum-check tails with ~1000 polling blocks)
  while ((f = __hip_atomic_load(&chal->flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) != seq && f != SC_CANCEL) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > 500000000ull) {  // 5 s: the host is gone or failed
      f = SC_CANCEL;
      __hip_atomic_store(&res->wait_expired, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  if (f == seq) {
#pragma unroll
    for (int j = 0; j < 8; j++)
      rd->r.v[j] = __hip_atomic_load(&chal->r.v[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    rd->abort = 0;
  } else {
    rd->abort = 1;
  }
}

// sum nb blocks' 4-vectors of partials in one block, write them and the flag to the host
__device__ void sc_last_block_publish(const Fr *__restrict__ partials, unsigned nb, Fr *lds, unsigned *counter,
                                      ScResult *res, uint32_t seq) {
  Fr b[4] = {Fr::zero(), Fr::zero(), Fr::zero(), Fr::zero()};
  for (unsigned bb = threadIdx.x; bb < nb; bb += blockDim.x)
#pragma unroll
    for (int x = 0; x < 4; x++) b[x] = add(b[x], partials[4 * (size_t)bb + x]);
  block_sum_fr<4>(b, lds);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int x = 0; x < 4; x++) res->sums[x] = b[x];
    *counter = 0;  // ready for the next launch (stream order)
    __threadfence_system();
    __hip_atomic_store(&res->flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// One sum-check round of a composition over K tables.
// FOLD:  tables in[] have 4P entries; bind r into out[] (2P entries), then sum the round values.
// !FOLD: tables in[] have 2P entries (round 0), just sum.
// Points X = 0, 1, 2, 3 (SKIP1: X = 1 is not formed -- from round 1 on the host takes g(1) as
// claim - g(0), src/sumcheck.rs:80-84; the prover checks the final value against the last claim).
// Each wave takes 64 consecutive pairs s at a time; the points are a loop over one inlined copy of
// the composition (v walks the line f0 + X (f1 - f0)): a quarter of the code of four unrolled
// copies, 3-4 % faster.  Each block's four sums go to partials[]; the last block to finish
// (counter) adds them up and publishes them to the host with `seq` as the flag.
template <bool FOLD, int K, bool SKIP1>
__global__ void __launch_bounds__(256, K <= 3 ? TNS_SC_WAVES3 : 2)
    k_sc_round_poly(ScTables t, const ScPoly *__restrict__ qp, size_t P, const ScRDev *rd, Fr *__restrict__ partials,
                    unsigned *counter, ScResult *res, uint32_t seq) {
  __shared__ Fr lds[4 * 16];
  __shared__ int last;
  if (FOLD && rd->abort) return;  // (the challenge never came: the host has given up on this proof)
  const Fr r = FOLD ? rd->r : Fr::zero();
  const int lane = threadIdx.x & 63;
  const ScPoly &q = *qp;  // device memory, uniform: scalar loads (a 1.2 KB kernarg spilled SGPRs)
  Fr acc0 = Fr::zero(), acc1 = Fr::zero(), acc2 = Fr::zero(), acc3 = Fr::zero();
  const size_t wstride = (size_t)gridDim.x * blockDim.x;
  for (size_t base = blockIdx.x * (size_t)blockDim.x + (threadIdx.x & ~63u); base < P; base += wstride) {
    const bool live = base + lane < P;  // (wave-uniform trip count)
    Fr v[K], d[K];
#pragma unroll
    for (int i = 0; i < K; i++) {
      if (FOLD) {  // (lazy folds: the next round and k_sc_final read [0, 2M] values)
        const Fr *p = t.in[i] + 4 * (base + (live ? lane : 0));
        const Fr x0 = p[0], x1 = p[1], x2 = p[2], x3 = p[3];
        v[i] = add2_dev(x0, mul_lazy_dev(r, sub2_dev(x1, x0)));
        d[i] = add2_dev(x2, mul_lazy_dev(r, sub2_dev(x3, x2)));
        if (live) {  // (64 contiguous bytes a lane; the stores merge in L2)
          t.out[i][2 * (base + lane)] = v[i];
          t.out[i][2 * (base + lane) + 1] = d[i];
        }
      } else {
        const Fr *p = t.in[i] + 2 * (base + (live ? lane : 0));
        v[i] = p[0];
        d[i] = p[1];
      }
      d[i] = sub2_dev(d[i], v[i]);
    }
    // (every lane evaluates -- no divergent branch around the products; a lane past the last row
    // adds zero)
    const Fr zero = Fr::zero();
#pragma unroll 1
    for (int x = 0; x < 4; x++) {
      if (!(SKIP1 && x == 1)) {
        const Fr e = sc_eval<K>(q, v);
        const Fr ez = live ? e : zero;
        if (x == 0) acc0 = add2_dev(acc0, ez);
        else if (x == 1) acc1 = add2_dev(acc1, ez);
        else if (x == 2) acc2 = add2_dev(acc2, ez);
        else acc3 = add2_dev(acc3, ez);
      }
      if (x < 3) {
#pragma unroll
        for (int i = 0; i < K; i++) v[i] = add2_dev(v[i], d[i]);
      }
    }
  }
  Fr a[4] = {sc_canon(acc0), sc_canon(acc1), sc_canon(acc2), sc_canon(acc3)};
  block_sum_fr<4>(a, lds);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int x = 0; x < 4; x++) partials[4 * (size_t)blockIdx.x + x] = a[x];
    __threadfence();
    last = atomicAdd(counter, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();  // every block's partials (each fenced before its increment) are visible
  sc_last_block_publish(partials, gridDim.x, lds, counter, res, seq);
}

// A small round (P pairs, latency-bound: one pair's folds and points in one lane is a chain of
// 4-12 dependent products, ~20 us at one wave per SIMD): four lanes per pair.  Lane x < K folds
// table x's two entries, the four lanes exchange the folded values (shuffles), and lane x
// evaluates the composition at point X = x -- a chain of 2 folds + 1 point instead of 2K folds +
// 3-4 points.  Sums per point: lanes x, x + 4, ... of each wave, then across the grid as in
// k_sc_round_poly (one-wave workgroups).
// one sweep of a round over pairs [0, P), 16 pairs per wave-iteration from pair 16 * blk with a
// stride of 16 * nblk; returns lane x's sum at point x (lanes x, x + 4, ... added: lane x < 4)
template <bool FOLD, int K, bool SKIP1>
__device__ __forceinline__ Fr sc_split_sweep(const ScTables &t, const ScPoly &q, size_t P, const Fr &r, size_t blk,
                                             size_t nblk) {
  const int lane = threadIdx.x & 63, x = lane & 3;
  const Fr zero = Fr::zero();
  const Fr *src = t.in[0];
  Fr *dst = t.out[0];
#pragma unroll
  for (int i = 1; i < K; i++)
    if (x == i) {
      src = t.in[i];
      dst = t.out[i];
    }
  Fr acc = zero;
  for (size_t base = blk * 16; base < P; base += nblk * 16) {  // (wave-uniform)
    const size_t s = base + (lane >> 2);
    const bool live = s < P;
    const size_t sl = live ? s : 0;
    Fr mv = zero, md = zero;  // this lane's table at the pair: the folded (or round-0) pair
    if (x < K) {
      if (FOLD) {
        const Fr *p = src + 4 * sl;
        const Fr x0 = p[0], x1 = p[1], x2 = p[2], x3 = p[3];
        mv = add2_dev(x0, mul_lazy_dev(r, sub2_dev(x1, x0)));
        md = add2_dev(x2, mul_lazy_dev(r, sub2_dev(x3, x2)));
        if (live) {
          dst[2 * s] = mv;
          dst[2 * s + 1] = md;
        }
      } else {
        mv = src[2 * sl];
        md = src[2 * sl + 1];
      }
      md = sub2_dev(md, mv);
    }
    Fr w[K];
#pragma unroll
    for (int i = 0; i < K; i++) {
      const int from = (lane & ~3) | i;
      Fr vi, di;
#pragma unroll
      for (int j = 0; j < 8; j++) {
        vi.v[j] = __shfl(mv.v[j], from, 64);
        di.v[j] = __shfl(md.v[j], from, 64);
      }
      w[i] = vi;  // the table's line at X = x: v + x d
#pragma unroll
      for (int j = 0; j < 3; j++)
        if (j < x) w[i] = add2_dev(w[i], di);
    }
    if (!(SKIP1 && x == 1)) {
      const Fr e = sc_eval<K>(q, w);
      acc = add2_dev(acc, live ? e : zero);
    }
  }
  acc = sc_canon(acc);
#pragma unroll
  for (int dd = 32; dd >= 4; dd >>= 1) {  // lanes x, x + 4, ...: lane x ends with point x's sum
    const Fr o = shfl_down_fr(acc, dd);
    if (lane + dd < 64) acc = add(acc, o);
  }
  return acc;
}

// a one-wave block's four point sums to partials[], and the last block of the grid to finish
// adds them up and publishes them (sc_last_block_publish)
__device__ __forceinline__ void sc_split_finish(const Fr &acc, Fr *__restrict__ partials, unsigned *counter,
                                                ScResult *res, uint32_t seq, Fr *lds, int *last) {
  const int lane = threadIdx.x;
  if (lane < 4) {
    partials[4 * (size_t)blockIdx.x + lane] = acc;
    __threadfence();
  }
  __syncthreads();
  if (lane == 0) *last = atomicAdd(counter, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!*last) return;
  __threadfence();  // every block's partials (each fenced before its increment) are visible
  sc_last_block_publish(partials, gridDim.x, lds, counter, res, seq);
}

template <bool FOLD, int K, bool SKIP1>
__global__ void __launch_bounds__(64) k_sc_round_split(ScTables t, const ScPoly *__restrict__ qp, size_t P,
                                                       const ScRDev *rd, Fr *__restrict__ partials, unsigned *counter,
                                                       ScResult *res, uint32_t seq) {
  __shared__ Fr lds[4 * 16];
  __shared__ int last;
  if (FOLD && rd->abort) return;
  const Fr r = FOLD ? rd->r : Fr::zero();
  const Fr acc = sc_split_sweep<FOLD, K, SKIP1>(t, *qp, P, r, blockIdx.x, gridDim.x);
  sc_split_finish(acc, partials, counter, res, seq, lds, &last);
}

// The small rounds' tail in one persistent launch (rounds r0 .. nv - 1 and the final fold): a
// round kernel per round pays two launch gaps (~5.6 us each) around the host's turn; here the
// grid stays resident and block 0 polls the host's challenge flag, relaying each challenge to the
// other blocks through device memory (ScTailSync: one agent-scope release per round).  The
// round's sums leave exactly as in k_sc_round_split (last block to finish publishes to the
// host), and the host's next challenge -- which it can only write after reading those sums --
// orders every block's table writes of this round before any block's reads in the next.
// Tables: round rr reads bufB (rr even) / bufC (rr odd) and writes the other; rr >= 2.
struct ScTailSync {
  uint32_t rflag;   // rounds whose challenge is in r[] (relayed by block 0)
  uint32_t abort;   // block 0 saw SC_CANCEL or its 5 s bound: every block returns
  uint32_t pad[14];
  Fr r[64];
};
struct ScPing {
  Fr *B[MAX_SC_TABLES], *C[MAX_SC_TABLES];
};

// block 0 thread 0: the host's challenge for `seq`, else false (cancel / 5 s: res->wait_expired)
__device__ bool sc_poll_host(ScChal *chal, uint32_t seq, Fr &r, ScResult *res) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
  uint32_t f;
  while ((f = __hip_atomic_load(&chal->flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) != seq) {
    if (f == SC_CANCEL) return false;
    if (__builtin_amdgcn_s_memrealtime() - t0 > 500000000ull) {
      __hip_atomic_store(&res->wait_expired, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // (r itself is read with system-scope loads below)
#pragma unroll
  for (int j = 0; j < 8; j++) r.v[j] = __hip_atomic_load(&chal->r.v[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return true;
}

// Rounds of <= SC_SOLO_PAIRS pairs run on block 0 alone: the grid-wide handoff of a round (the
// challenge relayed through device memory, every block's partials, the last-block count) costs a
// fixed ~13 us whatever the round's size (TNS_SC_TRACE, profiles/r06_sc_tail_trace.txt), while one
// wave sweeps 64 pairs in ~4 passes.
#ifndef TNS_SC_SOLO_PAIRS
#define TNS_SC_SOLO_PAIRS 64
#endif
constexpr size_t SC_SOLO_PAIRS = TNS_SC_SOLO_PAIRS;

// The last rounds, from the first of <= SC_HOST_PAIRS pairs, run on the host: the tail folds the
// tables once more (by that round's r) into mapped host memory and ends, and the host sweeps the
// few remaining pairs (4 x u64 arithmetic, hostfield.hpp) between its own transcript steps instead
// of a device round trip per round (~13 us each, profiles/r06_sc_tail_trace.txt).  0 disables.
#ifndef TNS_SC_HOST_PAIRS
#define TNS_SC_HOST_PAIRS 64
#endif
constexpr size_t SC_HOST_PAIRS = TNS_SC_HOST_PAIRS;  // (the hand-over round runs on block 0 alone)

// TNS_SC_TRACE builds (diagnostics, tools/sc_trace.py): the persistent tail records, per round, when
// block 0 starts waiting for the challenge, when it has it and when the last block publishes the
// round's sums (s_memrealtime, 100 MHz) into mapped host memory; the host adds its own turn times
#ifndef TNS_SC_TRACE
#define TNS_SC_TRACE 0
#endif
__device__ uint64_t *g_sc_trace = nullptr;

template <int K>
__global__ void __launch_bounds__(64) k_sc_tail(ScPing pp, const ScPoly *__restrict__ qp, unsigned r0, unsigned nv,
                                                size_t n, ScChal *chal, uint32_t chal_base, ScResult *res,
                                                uint32_t seq_base, Fr *__restrict__ partials, unsigned *counter,
                                                ScTailSync *sync, unsigned rh, Fr *__restrict__ htab) {
  __shared__ Fr lds[4 * 16];
  __shared__ int last;
  __shared__ Fr r_s;
  __shared__ int ok_s;
  const ScPoly &q = *qp;
  for (unsigned rr = r0; rr <= nv; rr++) {
    const unsigned t = rr - r0;
    const bool solo = rr >= rh || (n >> (rr + 1)) <= SC_SOLO_PAIRS;
    if (solo && blockIdx.x != 0) return;  // (the final fold / hand-over and the smallest rounds are block 0's)
    if (threadIdx.x == 0) {  // r_{rr - 1}
      bool ok = true;
      Fr r;
      if (blockIdx.x == 0) {
#if TNS_SC_TRACE
        if (g_sc_trace) g_sc_trace[4 * t] = __builtin_amdgcn_s_memrealtime();
#endif
        ok = sc_poll_host(chal, chal_base + rr, r, res);
#if TNS_SC_TRACE
        if (g_sc_trace) g_sc_trace[4 * t + 1] = __builtin_amdgcn_s_memrealtime();
#endif
        if (ok) {
          sync->r[t] = r;
          __hip_atomic_store(&sync->rflag, t + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          __hip_atomic_store(&sync->abort, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
      } else {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(&sync->rflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < t + 1) {
          if (__hip_atomic_load(&sync->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
              __builtin_amdgcn_s_memrealtime() - t0 > 600000000ull) {
            ok = false;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // (once: the tables and r[] of this round)
        if (ok) r = sync->r[t];
      }
      ok_s = ok;
      if (ok) r_s = r;
    }
    __syncthreads();
    if (!ok_s) return;
    const Fr r = r_s;
    ScTables tt{};
#pragma unroll
    for (int m = 0; m < K; m++) {  // round rr: in = bufB (rr even) / bufC (rr odd), out = the other
      tt.in[m] = rr % 2 == 0 ? pp.B[m] : pp.C[m];
      tt.out[m] = rr % 2 == 0 ? pp.C[m] : pp.B[m];
    }
    if (rr == rh && rh < nv) {  // hand-over: the tables folded by r_{rh-1} (K x L, kernel order) to the host
      const size_t L = n >> rr;
#pragma unroll
      for (int m = 0; m < K; m++) {
        const Fr *p = tt.in[m];
        for (size_t s = threadIdx.x; s < L; s += 64) {
          const Fr p0 = sc_canon(p[2 * s]), p1 = sc_canon(p[2 * s + 1]);
          htab[(size_t)m * L + s] = add(p0, mul(r, sub(p1, p0)));
        }
      }
      __threadfence_system();
      __syncthreads();
      if (threadIdx.x == 0) __hip_atomic_store(&res->flag, seq_base + t, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    if (rr == nv) {  // the final fold: in holds the last round's 2-entry tables
      if (blockIdx.x == 0) {
        if (threadIdx.x < (unsigned)K) {
          const Fr *p = tt.in[threadIdx.x];
          const Fr p0 = sc_canon(p[0]), p1 = sc_canon(p[1]);
          res->sums[threadIdx.x] = add(p0, mul(r, sub(p1, p0)));
          __threadfence_system();
        }
        __syncthreads();
        if (threadIdx.x == 0) {
          __threadfence_system();
          __hip_atomic_store(&res->flag, seq_base + t, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
      return;
    }
    const size_t P = n >> (rr + 1);
    if (solo) {  // block 0 sweeps every pair and publishes its own four sums
      const Fr acc = sc_split_sweep<true, K, true>(tt, q, P, r, 0, 1);
      if (threadIdx.x < 4) res->sums[threadIdx.x] = acc;
      __threadfence_system();  // (also this round's table writes, read by other lanes next round)
      __syncthreads();
      if (threadIdx.x == 0) __hip_atomic_store(&res->flag, seq_base + t, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
#if TNS_SC_TRACE
      if (threadIdx.x == 0 && g_sc_trace) g_sc_trace[4 * t + 2] = __builtin_amdgcn_s_memrealtime();
#endif
      __syncthreads();
      continue;
    }
    const Fr acc = sc_split_sweep<true, K, true>(tt, q, P, r, blockIdx.x, gridDim.x);
    sc_split_finish(acc, partials, counter, res, seq_base + t, lds, &last);
#if TNS_SC_TRACE
    if (last && threadIdx.x == 0 && g_sc_trace) g_sc_trace[4 * t + 2] = __builtin_amdgcn_s_memrealtime();
#endif
    __syncthreads();  // (ok_s / r_s are rewritten by thread 0 next round)
  }
}

// the last variable: table i's final value T[0] + r (T[1] - T[0]) (or T[0] when !FOLD), to the host
__global__ void __launch_bounds__(64) k_sc_final(ScTables t, int k, const ScRDev *rd, int fold, ScResult *res, uint32_t seq) {
  if (fold && rd->abort) return;
  const Fr r = fold ? rd->r : Fr::zero();
  if (threadIdx.x < (unsigned)k) {
    const Fr *p = t.in[threadIdx.x];
    const Fr p0 = sc_canon(p[0]), p1 = fold ? sc_canon(p[1]) : p0;  // (lazy round-kernel folds)
    res->sums[threadIdx.x] = fold ? add(p0, mul(r, sub(p1, p0))) : p0;
    __threadfence_system();
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(&res->flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Closure-free sum-check (no composition terms: every round polynomial is zero, so the
// challenges never wait for the device): the last m folds of the chain in one workgroup.
// Tables of 2^m entries in a[]; fold j binds ch[j] (LSB first, as k_sc_fold) and ping-pongs
// a -> b -> a ...; out[i] = table i bound at all m challenges.  Replaces m - 1 small
// k_sc_fold launches and the k final k_mle_fold launches (each ~20 us of launch gap).
struct ScTail {
  const Fr *a[MAX_SC_TABLES];  // first input (may be the caller's table: only read)
  Fr *b[MAX_SC_TABLES], *c[MAX_SC_TABLES];  // fold 0 -> b, then c, b, c, ...
};
constexpr unsigned SC_TAIL_LOG = 12;  // tables of <= 2^12 entries fold in the tail kernel

__global__ void __launch_bounds__(1024) k_sc_fold_tail(ScTail t, int k, int m, const Fr *__restrict__ ch,
                                                       Fr *__restrict__ out) {
  for (int j = 0; j < m; j++) {
    const Fr r = ch[j];
    const unsigned half = 1u << (m - 1 - j);
    for (int i = 0; i < k; i++) {
      const Fr *in = j == 0 ? t.a[i] : (j & 1) ? t.b[i] : t.c[i];
      Fr *o = (j & 1) ? t.c[i] : t.b[i];
      for (unsigned s = threadIdx.x; s < half; s += blockDim.x) {
        const Fr x0 = in[2 * s], x1 = in[2 * s + 1];
        o[s] = add(x0, mul(r, sub(x1, x0)));
      }
    }
    __syncthreads();  // fold j's outputs are fold j+1's inputs (other threads' entries)
  }
  if (threadIdx.x == 0)
    for (int i = 0; i < k; i++) out[i] = ((m - 1) & 1 ? t.c[i] : t.b[i])[0];
}


// The zero-constraint sum-check of Twist / Shout (src/twist.rs:186-214, src/shout.rs:160-184):
// every round polynomial is [0, 0, 0, 0], so the transcript alone yields the challenges and the
// host has all of them before any fold runs.  The fold chain by those challenges is then pure
// device work with no host wait: launched on `st` (a side stream) it runs under the openings,
// and the k tables bound at every challenge land in d_out.  The input tables are only read.
// three zero-closure folds in one pass (challenges r0, r1, r2 of consecutive rounds): out[s] from
// in[8s .. 8s + 7] -- one read of the tables per three rounds instead of per round
// flags (optional): the last table is 0/1 flags given as bytes (entries >= n_flags are 0), so its
// first fold is a select among 0, 1, r0 and 1 - r0 -- the table itself never exists
__global__ void __launch_bounds__(256) k_sc_fold3(ScTables t, int k, size_t P, Fr r0, Fr r1, Fr r2,
                                                  const uint8_t *__restrict__ flags, size_t n_flags) {
  const Fr one = Fr::one(), omr = sub(Fr::one(), r0);
  for (size_t s = blockIdx.x * (size_t)blockDim.x + threadIdx.x; s < P; s += (size_t)gridDim.x * blockDim.x) {
#pragma unroll
    for (int i = 0; i < MAX_SC_TABLES; i++) {
      if (i < k) {
        Fr a[4];
        if (flags && i == k - 1) {
          uint32_t f[8];
          if (8 * s + 8 <= n_flags && ((uintptr_t)flags & 7) == 0) {
            const uint2 w = *reinterpret_cast<const uint2 *>(flags + 8 * s);  // 8-byte aligned
#pragma unroll
            for (int j = 0; j < 4; j++) {
              f[j] = (w.x >> (8 * j)) & 0xff;
              f[4 + j] = (w.y >> (8 * j)) & 0xff;
            }
          } else {
#pragma unroll
            for (int j = 0; j < 8; j++) f[j] = 8 * s + j < n_flags ? flags[8 * s + j] : 0u;
          }
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const bool f0 = f[2 * j] != 0, f1 = f[2 * j + 1] != 0;  // f0 + r0 (f1 - f0)
            a[j] = f0 ? (f1 ? one : omr) : (f1 ? r0 : Fr::zero());
          }
        } else {
          const Fr *p = t.in[i] + 8 * s;
          Fr x[8];
#pragma unroll
          for (int j = 0; j < 8; j++) x[j] = p[j];
#pragma unroll
          for (int j = 0; j < 4; j++) a[j] = add(x[2 * j], mul(r0, sub(x[2 * j + 1], x[2 * j])));
        }
        const Fr b0 = add(a[0], mul(r1, sub(a[1], a[0]))), b1 = add(a[2], mul(r1, sub(a[3], a[2])));
        t.out[i][s] = add(b0, mul(r2, sub(b1, b0)));
      }
    }
  }
}

static unsigned sc_tail_round(unsigned nv) { return std::max(1u, nv + 1 - std::min(nv, SC_TAIL_LOG)); }

bool sumcheck_folds_take_flag_bytes(unsigned nv) { return sc_tail_round(nv) > 3; }

void sumcheck_zero_folds_async(Ctx *c, hipStream_t st, Fr *const *tables, int k, unsigned nv, const Fr *chal_pinned,
                               Fr *d_out, const uint8_t *flags, size_t n_flags) {
  if (k < 1 || k > MAX_SC_TABLES) throw Error(TNS_ERR_INVALID_PARAMETERS, "at most 4 sum-check tables");
  if (flags && !sumcheck_folds_take_flag_bytes(nv))
    throw Error(TNS_ERR_SUMCHECK, "flag bytes need a first three-round fold pass");
  if (nv == 0) {
    for (int i = 0; i < k; i++) TNS_HIP(hipMemcpyAsync(d_out + i, tables[i], sizeof(Fr), hipMemcpyDeviceToDevice, st));
    return;
  }
  const size_t n = (size_t)1 << nv;
  Fr *bufB[MAX_SC_TABLES], *bufC[MAX_SC_TABLES];
  for (int i = 0; i < k; i++) {
    bufB[i] = (Fr *)c->sc_half[i].ensure(sizeof(Fr) * (n / 2 + 1));
    bufC[i] = (Fr *)c->sc_pong[i].ensure(sizeof(Fr) * (n / 4 + 1));
  }
  Fr *d_ch = (Fr *)c->sc_chal.ensure(sizeof(Fr) * nv);
  TNS_HIP(hipMemcpyAsync(d_ch, chal_pinned, sizeof(Fr) * nv, hipMemcpyHostToDevice, st));
  // rounds 1 .. tail_rnd - 1 fold by r_{rnd-1} in k_sc_fold; the rest (tables of <= 2^12) in
  // one k_sc_fold_tail workgroup, down to one value per table
  const unsigned tail_rnd = sc_tail_round(nv);
  Fr *src[MAX_SC_TABLES], *dst[MAX_SC_TABLES];
  for (int i = 0; i < k; i++) {
    src[i] = tables[i];
    dst[i] = bufB[i];
  }
  Fr ch[64];
  std::memcpy(ch, chal_pinned, sizeof(Fr) * std::min(nv, 64u));
  bool first = true;
  for (unsigned rnd = 1; rnd < tail_rnd;) {
    ScTables tt{};
    for (int i = 0; i < k; i++) {
      tt.in[i] = src[i];
      tt.out[i] = dst[i];
    }
    if (rnd + 2 < tail_rnd) {  // rounds rnd .. rnd + 2 in one pass (one read of the tables per three rounds)
      const size_t P = n >> (rnd + 2);
      TNS_PROF_ON(c, st, "sumcheck_round", 288.0 * (double)P * k);
      k_sc_fold3<<<grid_for(P, 256, 4096), 256, 0, st>>>(tt, k, P, ch[rnd - 1], ch[rnd], ch[rnd + 1],
                                                          first ? flags : nullptr, n_flags);
      TNS_LAUNCH_CHECK();
      rnd += 3;
    } else {
      const size_t P = n >> (rnd + 1);
      TNS_PROF_ON(c, st, "sumcheck_round", 192.0 * (double)P * k);
      k_sc_fold<<<grid_for(P, 256, 2048), 256, 0, st>>>(tt, k, P, ch[rnd - 1]);
      TNS_LAUNCH_CHECK();
      rnd += 1;
    }
    for (int i = 0; i < k; i++) {
      if (first) {  // after the first pass: bufB holds the tables' fold
        src[i] = bufB[i];
        dst[i] = bufC[i];
      } else {
        std::swap(src[i], dst[i]);
      }
    }
    first = false;
  }
  ScTail tl{};
  for (int i = 0; i < k; i++) {
    tl.a[i] = src[i];
    tl.b[i] = dst[i];
    tl.c[i] = first ? bufC[i] : src[i];
  }
  const int m = (int)(nv - tail_rnd + 1);
  TNS_PROF_ON(c, st, "sumcheck_round", 96.0 * (double)(n >> (tail_rnd - 1)) * k);
  k_sc_fold_tail<<<1, 1024, 0, st>>>(tl, k, m, d_ch + (tail_rnd - 1), d_out);
  TNS_LAUNCH_CHECK();
}

// ---------------------------------------------------------------- generic sum-check, host side
// Waits for a round kernel's published result: polls the flag in fine-grained host memory (the
// last workgroup writes it); a flag that does not arrive within 30 s falls back to a stream
// synchronize, which reports any device error, and then fails.
static const ScResult &sc_wait(Ctx *c, uint32_t seq) {
  volatile ScResult *res = (volatile ScResult *)c->sc_mapped.p;
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned spin = 0; __atomic_load_n(&res->flag, __ATOMIC_ACQUIRE) != seq; spin++) {
    if (const uint32_t w = __atomic_load_n(&res->wait_expired, __ATOMIC_RELAXED)) {
      res->wait_expired = 0;
      throw Error(TNS_ERR_DEVICE, "sum-check: a device waiter gave up on challenge #" + std::to_string(w) +
                                      " after 5 s (the host's turn was too slow); its round did not run");
    }
    if ((spin & 1023) == 1023 &&
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > 30.0) {
      TNS_HIP(hipStreamSynchronize(c->stream));
      if (__atomic_load_n(&res->flag, __ATOMIC_ACQUIRE) == seq) break;
      throw Error(TNS_ERR_DEVICE, "sum-check round kernel did not publish its sums");
    }
  }
  return *(const ScResult *)c->sc_mapped.p;
}

struct ScRun {
  Ctx *c;
  int k;
  ScPoly q;
  int perm[MAX_SC_TABLES];  // kernel table m reads the caller's table perm[m]
  const ScPoly *q_dev;
  unsigned max_grid;
  Fr *partials;
  unsigned *counter;
  ScResult *res_dev;
  ScChal *chal;      // host view
  ScChal *chal_dev;  // device view
  ScRDev *rd;
};

static ScRun sc_run(Ctx *c, int k, const SumcheckTerm *terms, int n_terms, size_t max_blocks) {
  ScRun R{};
  R.c = c;
  R.k = k;
  R.q = sc_poly(terms, n_terms, k, R.perm);
  R.max_grid = (unsigned)std::max(1, c->num_cu) * 4;  // one round of resident blocks: threads loop over s
  ScPoly *qd = (ScPoly *)c->sc_poly.ensure(sizeof(ScPoly));
  ScPoly *qh = (ScPoly *)c->sc_poly_host.ensure(sizeof(ScPoly));  // pinned: outlives the async copy
  *qh = R.q;
  TNS_HIP(hipMemcpyAsync(qd, qh, sizeof(ScPoly), hipMemcpyHostToDevice, c->stream));
  R.q_dev = qd;
  // (sc_launch's grids: at most max_grid * 4 one-wave blocks)
  R.partials = (Fr *)c->scratch[6].ensure(sizeof(Fr) * 4 * std::max<size_t>(max_blocks, (size_t)R.max_grid * 4));
  R.counter = (unsigned *)c->sc_counter.ensure(sizeof(unsigned));
  // zero once per sum-check (each round's last workgroup leaves it zero for the next round)
  TNS_HIP(hipMemsetAsync(R.counter, 0, sizeof(unsigned), c->stream));
  c->sc_mapped.ensure(sizeof(ScResult));
  ((volatile ScResult *)c->sc_mapped.p)->wait_expired = 0;  // (nothing of an earlier call is still running)
  R.res_dev = (ScResult *)c->sc_mapped.dev;
  R.chal = (ScChal *)c->sc_handoff.ensure(sizeof(ScChal));
  R.chal_dev = (ScChal *)c->sc_handoff.dev;
  R.rd = (ScRDev *)c->sc_rdev.ensure(sizeof(ScRDev));
  TNS_HIP(hipMemsetAsync(R.rd, 0, sizeof(ScRDev), c->stream));
  return R;
}

// The generic sum-check's schedule (round 5, profiles/r05_ab_sumcheck.txt):
//  * rounds of <= 2^SC_SPLIT_LOG pairs run four lanes a pair (k_sc_round_split; 2^12-2^14 measured
//    alike, at 2^16 the pairs-per-lane kernel is 2x faster);
//  * the rounds of <= 2^SC_PTAIL_LOG pairs and the final fold run as one persistent launch of at
//    most SC_PTAIL_BLOCKS one-wave blocks (k_sc_tail; 64 beat 16-1024);
//  * each round's kernels are queued before its challenge exists (k_sc_wait_r).
#ifndef TNS_SC_SPLIT_LOG  // (build-time A/B only: tools/build_variant.sh)
#define TNS_SC_SPLIT_LOG 13
#endif
#ifndef TNS_SC_PTAIL_LOG
#define TNS_SC_PTAIL_LOG 13
#endif
constexpr unsigned SC_SPLIT_LOG = TNS_SC_SPLIT_LOG, SC_PTAIL_LOG = TNS_SC_PTAIL_LOG, SC_PTAIL_BLOCKS = 64;

// one round's launch (tables already in kernel order); returns the flag value to wait for
template <bool FOLD, bool SKIP1>
static uint32_t sc_launch(ScRun &R, const ScTables &tt, size_t P) {
  // small rounds: one-wave workgroups spread over many CUs (a round of 2^8 pairs on one 256-thread
  // workgroup ran 35 us: one CU's multiply rate), large rounds: one round of resident 256-thread
  // workgroups, each thread looping over pairs
  const uint32_t seq = ++R.c->sc_seq;
  hipStream_t st = R.c->stream;
  const size_t split_max = (size_t)1 << SC_SPLIT_LOG;
  if (P <= split_max) {  // four lanes a pair, 16 pairs a one-wave block (2^12-2^14 measured alike;
                         // at 2^16 the pairs-per-lane kernel is 2x faster)
    const unsigned g = grid_for(P, 16, R.max_grid * 4);
#define TNS_SC_K(K) \
  k_sc_round_split<FOLD, K, SKIP1><<<g, 64, 0, st>>>(tt, R.q_dev, P, R.rd, R.partials, R.counter, R.res_dev, seq)
    switch (R.k) {
      case 1: TNS_SC_K(1); break;
      case 2: TNS_SC_K(2); break;
      case 3: TNS_SC_K(3); break;
      default: TNS_SC_K(4); break;
    }
#undef TNS_SC_K
  } else {
    const unsigned bs = P >= ((size_t)1 << 16) ? 256u : 64u;
    const unsigned g = grid_for(P, bs, R.max_grid * (256 / bs));
#define TNS_SC_K(K) \
  k_sc_round_poly<FOLD, K, SKIP1><<<g, bs, 0, st>>>(tt, R.q_dev, P, R.rd, R.partials, R.counter, R.res_dev, seq)
    switch (R.k) {
      case 1: TNS_SC_K(1); break;
      case 2: TNS_SC_K(2); break;
      case 3: TNS_SC_K(3); break;
      default: TNS_SC_K(4); break;
    }
#undef TNS_SC_K
  }
  TNS_LAUNCH_CHECK();
  return seq;
}

static void sc_round_sums(ScRun &R, uint32_t seq, Fr e[4]) {
  const ScResult &res = sc_wait(R.c, seq);
  for (int x = 0; x < 4; x++) e[x] = res.sums[x];
}

// the composition at one point of the caller's table order (src/sumcheck.rs:104)
static Fr eval_composition_host(const Fr *vals, const SumcheckTerm *terms, int n_terms) {
  Fr s = Fr::zero();
  for (int t = 0; t < n_terms; t++) {
    Fr p = terms[t].coeff;
    for (int j = 0; j < 3; j++)
      if (terms[t].tab[j] >= 0) p = mul(p, vals[terms[t].tab[j]]);
    s = add(s, p);
  }
  return s;
}

// The sum-check's last rounds on the host (SC_HOST_PAIRS): the same sums as the device's round
// kernels -- g(X) = sum over pairs s of the composition at T[2s] + X (T[2s+1] - T[2s]), at X = 0, 2,
// 3 (g(1) is the claim minus g(0)) -- and the same fold T'[s] = T[2s] + r (T[2s+1] - T[2s])
// (src/sumcheck.rs:60-100), over tables in the caller's order
struct ScHostRounds {
  std::vector<HFr> t[MAX_SC_TABLES];
  struct Term {
    HFr coeff;
    int tab[3];
  };
  std::vector<Term> terms;
  int k = 0;
  void load(const Fr *src, int k_, size_t L, const int *perm, const SumcheckTerm *tm, int n_terms) {
    k = k_;
    for (int m = 0; m < k; m++) {  // (kernel table m is the caller's perm[m])
      std::vector<HFr> &v = t[perm[m]];
      v.resize(L);
      std::memcpy((void *)v.data(), (const void *)(src + (size_t)m * L), sizeof(Fr) * L);
    }
    terms.resize(n_terms);
    for (int i = 0; i < n_terms; i++) {
      terms[i].coeff = HFr::of(tm[i].coeff);
      for (int j = 0; j < 3; j++) terms[i].tab[j] = tm[i].tab[j];
    }
  }
  HFr comp(const HFr *v) const {
    HFr s = HFr::zero();
    for (const Term &tm : terms) {
      HFr p = tm.coeff;
      for (int j = 0; j < 3; j++)
        if (tm.tab[j] >= 0) p = p * v[tm.tab[j]];
      s = s + p;
    }
    return s;
  }
  void sums(Fr e[4]) const {
    const size_t P = t[0].size() / 2;
    HFr acc[3] = {HFr::zero(), HFr::zero(), HFr::zero()};
    for (size_t s = 0; s < P; s++) {
      HFr v[MAX_SC_TABLES], d[MAX_SC_TABLES];
      for (int i = 0; i < k; i++) {
        v[i] = t[i][2 * s];
        d[i] = t[i][2 * s + 1] - v[i];
      }
      acc[0] = acc[0] + comp(v);
      for (int x = 1; x < 3; x++) {  // X = 2, 3
        for (int i = 0; i < k; i++) v[i] = v[i] + (x == 1 ? h_dbl(d[i]) : d[i]);
        acc[x] = acc[x] + comp(v);
      }
    }
    e[0] = acc[0].fp();
    e[1] = Fr::zero();  // (the caller's: the claim minus g(0))
    e[2] = acc[1].fp();
    e[3] = acc[2].fp();
  }
  void fold(const Fr &r) {
    const HFr hr = HFr::of(r);
    for (int i = 0; i < k; i++) {
      std::vector<HFr> &v = t[i];
      const size_t h = v.size() / 2;
      for (size_t s = 0; s < h; s++) v[s] = v[2 * s] + hr * (v[2 * s + 1] - v[2 * s]);
      v.resize(h);
    }
  }
};

// sum over {0,1}^nv of the composition (the honest prover's claimed sum): round 0's sums at
// X = 0 and X = 1, added
Fr composition_sum_dev(Ctx *c, Fr *const *tables, int k, unsigned nv, const SumcheckTerm *terms, int n_terms) {
  if (k < 1 || k > MAX_SC_TABLES) throw Error(TNS_ERR_INVALID_PARAMETERS, "1 to 4 sum-check tables");
  if (nv == 0) {
    Fr v[MAX_SC_TABLES];
    for (int i = 0; i < k; i++) TNS_HIP(hipMemcpyAsync(&v[i], tables[i], sizeof(Fr), hipMemcpyDeviceToHost, c->stream));
    TNS_HIP(hipStreamSynchronize(c->stream));
    return eval_composition_host(v, terms, n_terms);
  }
  const size_t P = (size_t)1 << (nv - 1);
  ScRun R = sc_run(c, k, terms, n_terms, grid_for(P, 256, 2048));
  ScTables tt{};
  for (int m = 0; m < k; m++) tt.in[m] = tables[R.perm[m]];
  Fr e[4];
  sc_round_sums(R, sc_launch<false, false>(R, tt, P), e);
  return add(e[0], e[1]);
}

// SumCheck::prove for a composition with terms over k >= 1 tables (sumcheck_prove_dev's main
// case).  Round rr + 1's kernels are queued while round rr runs -- k_sc_wait_r, then the round
// kernel -- so the host's part of a round (read the sums, interpolate, transcript, challenge) is
// the only gap between two round kernels: the kernel launch latency (~15 us a round) leaves the
// critical path.
static void sumcheck_prove_terms(Ctx *c, Fr *const *tables, int k, unsigned nv, const Fr &claimed,
                                 const SumcheckTerm *terms, int n_terms, HostTranscript &tr, Fr *rounds,
                                 Fr *challenges, Fr *final_vals, Fr *final_eval) {
  const size_t n = (size_t)1 << nv;
  Fr *bufB[MAX_SC_TABLES], *bufC[MAX_SC_TABLES];
  for (int i = 0; i < k; i++) {
    bufB[i] = (Fr *)c->scratch[2 + i].ensure(sizeof(Fr) * (n / 2 + 1));
    bufC[i] = (Fr *)c->sc_pong[i].ensure(sizeof(Fr) * (n / 4 + 1));
  }
  ScRun R = sc_run(c, k, terms, n_terms, grid_for(n / 2 + 1, 256, 2048));
  // round rr reads the caller's tables (rr <= 1) or the previous round's output and writes the
  // folded tables into bufB (rr odd) / bufC (rr even >= 2): the caller's tables stay intact
  auto in_of = [&](unsigned rr, int m) -> Fr * {
    return rr <= 1 ? tables[R.perm[m]] : (rr % 2 == 0 ? bufB[R.perm[m]] : bufC[R.perm[m]]);
  };
  auto out_of = [&](unsigned rr, int m) -> Fr * { return rr % 2 == 1 ? bufB[R.perm[m]] : bufC[R.perm[m]]; };
  const uint32_t chal_base = c->sc_chal_seq;
  c->sc_chal_seq += nv + 1;
  R.chal->flag = 0;  // (no stale value can match: chal_base + i is fresh)
  // the persistent tail (k_sc_tail) from the first round r0 >= 2 of <= 2^SC_PTAIL_LOG pairs
  unsigned r0 = nv;
  for (unsigned rr = 2; rr < nv; rr++)
    if ((n >> (rr + 1)) <= ((size_t)1 << SC_PTAIL_LOG)) {
      r0 = rr;
      break;
    }
  const bool tail = r0 < nv;
  // the host's rounds: rh .. nv - 1 (rh == nv: none; the tail's final fold gives the values)
  unsigned rh = nv;
  for (unsigned rr = r0; tail && rr < nv; rr++)
    if ((n >> (rr + 1)) <= SC_HOST_PAIRS) {
      rh = rr;
      break;
    }
  Fr *htab_dev = nullptr;
  if (rh < nv) {
    c->sc_htab.ensure(sizeof(Fr) * k * (n >> rh));
    htab_dev = (Fr *)c->sc_htab.dev;
  }
  uint32_t tail_seq = 0;
  // queue round rr (rr >= 1: behind the wait for challenge r_{rr-1}); rr == nv: the final fold
  auto queue = [&](unsigned rr) -> uint32_t {
    if (tail && rr >= r0) {  // rounds r0 .. nv - 1 and the final fold: one launch at r0
      if (rr == r0) {
        ScTailSync *sync = (ScTailSync *)c->sc_tail_sync.ensure(sizeof(ScTailSync));
        TNS_HIP(hipMemsetAsync(sync, 0, sizeof(ScTailSync), c->stream));
        ScPing pp{};
        for (int m = 0; m < k; m++) {
          pp.B[m] = bufB[R.perm[m]];
          pp.C[m] = bufC[R.perm[m]];
        }
        tail_seq = c->sc_seq + 1;
        c->sc_seq += nv - r0 + 1;
        const unsigned g = (unsigned)std::min<size_t>(SC_PTAIL_BLOCKS, std::max<size_t>(1, (n >> (r0 + 1)) / 16));
#define TNS_SC_K(K)                                                                                             \
  k_sc_tail<K><<<g, 64, 0, c->stream>>>(pp, R.q_dev, r0, nv, n, R.chal_dev, chal_base, R.res_dev, tail_seq, \
                                       R.partials, R.counter, sync, rh, htab_dev)
        switch (k) {
          case 1: TNS_SC_K(1); break;
          case 2: TNS_SC_K(2); break;
          case 3: TNS_SC_K(3); break;
          default: TNS_SC_K(4); break;
        }
#undef TNS_SC_K
        TNS_LAUNCH_CHECK();
      }
      return tail_seq + (rr - r0);
    }
    if (rr > 0) {
      k_sc_wait_r<<<1, 64, 0, c->stream>>>(R.chal_dev, chal_base + rr, R.rd, R.res_dev);
      TNS_LAUNCH_CHECK();
    }
    ScTables tt{};
    if (rr == nv) {
      // nv <= 1: the caller's tables (nv == 0 reads them as they are; nv - 1 would wrap)
      for (int m = 0; m < k; m++) tt.in[m] = nv <= 1 ? tables[R.perm[m]] : out_of(nv - 1, m);
      const uint32_t seq = ++c->sc_seq;
      k_sc_final<<<1, 64, 0, c->stream>>>(tt, k, R.rd, nv > 0, R.res_dev, seq);
      TNS_LAUNCH_CHECK();
      return seq;
    }
    const size_t P = n >> (rr + 1);
    for (int m = 0; m < k; m++) {
      tt.in[m] = in_of(rr, m);
      tt.out[m] = out_of(rr, m);
    }
    TNS_PROF(c, "sumcheck_round", (rr == 0 ? 64.0 : 192.0) * (double)P * k);  // (the round kernel alone)
    return rr == 0 ? sc_launch<false, false>(R, tt, P) : sc_launch<true, true>(R, tt, P);
  };
  auto publish = [&](unsigned i, const Fr &ch) {  // challenge r_i for the kernels waiting on it
    R.chal->r = ch;
    __atomic_store_n(&R.chal->flag, chal_base + i + 1, __ATOMIC_RELEASE);
  };
#if TNS_SC_TRACE
  static MappedHostBuf trace_buf;
  uint64_t *trace_h = (uint64_t *)trace_buf.ensure(4 * 64 * sizeof(uint64_t));
  std::memset(trace_h, 0, 4 * 64 * sizeof(uint64_t));
  uint64_t *trace_d = (uint64_t *)trace_buf.dev;
  TNS_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_sc_trace), &trace_d, sizeof trace_d, 0, hipMemcpyHostToDevice, c->stream));
  std::vector<double> t_seen(nv + 1, 0.0), t_pub(nv + 1, 0.0);
  const auto tt0 = std::chrono::steady_clock::now();
  auto us = [&]() { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tt0).count(); };
#endif
  try {
    Fr cur = claimed;
    char lab[64];
    uint32_t seq = queue(0);  // (nv == 0: the final kernel, reading the tables as they are)
    if (nv > 0) tr.prehash(tr.state.size() + strlen("sumcheck_round_0") + 4 * 32 + strlen("sumcheck_challenge_0"));
    ScHostRounds H;  // (rounds rh .. nv - 1)
    for (unsigned rnd = 0; rnd < nv; rnd++) {
      const uint32_t seq_next = rnd + 1 <= rh ? queue(rnd + 1) : 0;  // (rnd + 1 == rh: the hand-over)
      Fr e[4];
      if (rnd < rh) {
        sc_round_sums(R, seq, e);
      } else {
        if (rnd == rh) {
          sc_wait(c, seq);
          H.load((const Fr *)c->sc_htab.p, k, n >> rh, R.perm, terms, n_terms);
        }
        H.sums(e);
      }
#if TNS_SC_TRACE
      t_seen[rnd] = us();
#endif
      if (rnd > 0) e[1] = sub(cur, e[0]);  // (SKIP1 rounds; round 0 forms g(1) and checks the claim)
      Fr coeffs[4];
      interpolate4_host(e, coeffs);  // lagrange_interpolate of 4 points (src/sumcheck.rs:201-206)
      if (add(horner_host(coeffs, 4, Fr::zero()), horner_host(coeffs, 4, Fr::one())) != cur) {  // :80-84
        snprintf(lab, sizeof lab, "Round %u consistency check failed", rnd);
        throw Error(TNS_ERR_SUMCHECK, lab);
      }
      for (int x = 0; x < 4; x++) rounds[4 * rnd + x] = coeffs[x];
      snprintf(lab, sizeof lab, "sumcheck_round_%u", rnd);  // src/sumcheck.rs:90-96
      tr.append_label(lab);
      for (int x = 0; x < 4; x++) tr.append_fr(coeffs[x]);
      snprintf(lab, sizeof lab, "sumcheck_challenge_%u", rnd);
      const Fr ch = tr.challenge(lab);
      if (rnd < rh) publish(rnd, ch);  // (first: the device's next round waits for it)
      else H.fold(ch);
#if TNS_SC_TRACE
      t_pub[rnd] = us();
#endif
      if (challenges) challenges[rnd] = ch;
      cur = horner_host(coeffs, 4, ch);
      seq = seq_next;
      if (rnd + 1 < nv) {  // the next challenge's hash over the state so far, while the device works
        char l1[64], l2[64];
        const int n1 = snprintf(l1, sizeof l1, "sumcheck_round_%u", rnd + 1);
        const int n2 = snprintf(l2, sizeof l2, "sumcheck_challenge_%u", rnd + 1);
        tr.prehash(tr.state.size() + (size_t)n1 + 4 * 32 + (size_t)n2);
      }
    }
    const ScResult &res = rh < nv ? *(const ScResult *)c->sc_mapped.p : sc_wait(c, seq);
#if TNS_SC_TRACE
    t_seen[nv] = us();
    for (unsigned rnd = 0; rnd < nv; rnd++)
      fprintf(stderr, "[sc-trace] round %2u host: sums seen %9.1f us, challenge out %9.1f us (turn %5.1f us)%s\n", rnd,
              t_seen[rnd], t_pub[rnd], t_pub[rnd] - t_seen[rnd], rnd >= r0 ? " [tail]" : "");
    fprintf(stderr, "[sc-trace] final seen %9.1f us\n", t_seen[nv]);
    for (unsigned t = 0; tail && r0 + t < nv; t++) {
      const uint64_t *d = trace_h + 4 * t, *dn = trace_h + 4 * (t + 1);
      const double wait = (d[1] - d[0]) * 0.01, comp = (d[2] - d[1]) * 0.01;
      const double turn = (r0 + t + 1 < nv && dn[1]) ? (dn[1] - d[2]) * 0.01 : -1;
      fprintf(stderr, "[sc-trace] tail round %2u (pairs %zu): device wait for r %7.1f us, compute+publish %7.1f us, "
                      "publish -> next r on device %7.1f us\n", r0 + t, n >> (r0 + t + 1), wait, comp, turn);
    }
    void *nullp = nullptr;
    TNS_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_sc_trace), &nullp, sizeof nullp));
#endif
    Fr vals[MAX_SC_TABLES];
    if (rh < nv) {
      for (int i = 0; i < k; i++) vals[i] = H.t[i][0].fp();
    } else {
      for (int m = 0; m < k; m++) vals[R.perm[m]] = res.sums[m];
    }
    for (int i = 0; i < k; i++) final_vals[i] = vals[i];
    *final_eval = eval_composition_host(vals, terms, n_terms);  // polynomial(&fixed_variables), :104
    // the last round's claim is g_{nv-1}(r_{nv-1}) = f(r): an honest prover's final value must
    // equal it; with g(1) taken from the claim (SKIP1) this is the check that catches a device
    // miscompute
    if (nv > 0 && *final_eval != cur)
      throw Error(TNS_ERR_SUMCHECK, "final evaluation does not match the last round's claim (device result inconsistent)");
  } catch (...) {
    // kernels may be queued behind a challenge that will never come: release them, then drain
    __atomic_store_n(&R.chal->flag, SC_CANCEL, __ATOMIC_RELEASE);
    (void)hipStreamSynchronize(c->stream);
    throw;
  }
}

// SumCheck::prove (src/sumcheck.rs:56-110) for an MLE composition.
// tables: k device arrays of 2^nv Fr (read only).  Host transcript drives challenges.
int sumcheck_prove_dev(Ctx *c, Fr *const *tables, int k, unsigned nv, const Fr &claimed,
                       const SumcheckTerm *terms, int n_terms, HostTranscript &tr, Fr *rounds,
                       Fr *challenges, Fr *final_vals, Fr *final_eval) {
  if (k < 0 || k > MAX_SC_TABLES) throw Error(TNS_ERR_INVALID_PARAMETERS, "at most 4 sum-check tables");
  const bool has_terms = n_terms > 0;
  if (has_terms && k > 0) {
    sumcheck_prove_terms(c, tables, k, nv, claimed, terms, n_terms, tr, rounds, challenges, final_vals, final_eval);
    return TNS_OK;
  }
  const size_t n = (size_t)1 << nv;
  // ping-pong: round r (r >= 1) reads src (2^(nv-r+1)) and writes dst (2^(nv-r)); round 1
  // reads the caller's tables, later rounds alternate between bufB and bufC, so the input
  // tables are left intact (Twist / Shout open the same evaluation vectors afterwards).
  Fr *bufB[MAX_SC_TABLES], *bufC[MAX_SC_TABLES];
  for (int i = 0; i < k; i++) {
    bufB[i] = (Fr *)c->scratch[2 + i].ensure(sizeof(Fr) * (n / 2 + 1));
    bufC[i] = (Fr *)c->sc_pong[i].ensure(sizeof(Fr) * (n / 4 + 1));
  }
  ScRun R = sc_run(c, k, terms, n_terms, grid_for(n / 2 + 1, 256, 2048));
  // kernel order m = caller's table perm[m] (the composition's cheapest nesting)
  Fr *src[MAX_SC_TABLES], *dst[MAX_SC_TABLES];
  for (int m = 0; m < k; m++) {
    src[m] = tables[R.perm[m]];
    dst[m] = bufB[R.perm[m]];
  }
  Fr cur = claimed, r_prev = Fr::zero();
  char lab[64];
  // closure-free chains hand their last folds to k_sc_fold_tail: from round `tail_rnd` on
  // (input tables of n >> (tail_rnd - 1) <= 2^SC_TAIL_LOG entries) only the transcript runs
  const unsigned tail_rnd =
      (!has_terms && k > 0 && nv >= 2) ? std::max(1u, nv + 1 - std::min(nv, SC_TAIL_LOG)) : nv + 1;
  Fr tail_ch[64];
  for (unsigned rnd = 0; rnd < nv; rnd++) {
    const size_t P = n >> (rnd + 1);  // output pairs of this round
    Fr e[4] = {Fr::zero(), Fr::zero(), Fr::zero(), Fr::zero()};
    if (rnd >= tail_rnd) {
      tail_ch[rnd - tail_rnd] = r_prev;  // this round's fold runs in k_sc_fold_tail
    } else {
      ScTables tt{};
      for (int m = 0; m < k; m++) {
        tt.in[m] = src[m];
        tt.out[m] = dst[m];
      }
      uint32_t seq = 0;
      {  // (the stage's HIP events bracket the launch alone, not the host's wait for its sums)
        TNS_PROF(c, "sumcheck_round", (rnd == 0 ? 64.0 : 192.0) * (double)P * k);
        if (rnd > 0 && k > 0) {  // (closure-free chain: folds only)
          k_sc_fold<<<grid_for(P, 256, 2048), 256, 0, c->stream>>>(tt, k, P, r_prev);
          TNS_LAUNCH_CHECK();
        }
      }
      if (seq) sc_round_sums(R, seq, e);
      if (has_terms && k == 0) {  // a constant composition: every point sums to c * P
        const Fr cP = mul(eval_composition_host(nullptr, terms, n_terms), from_u64<FrCfg>((uint64_t)P));
        for (int x = 0; x < 4; x++) e[x] = cP;
      }
      if (rnd > 0)  // src now holds the freshly folded 2P-entry tables
        for (int m = 0; m < k; m++) {
          if (rnd == 1) {
            src[m] = bufB[R.perm[m]];
            dst[m] = bufC[R.perm[m]];
          } else {
            std::swap(src[m], dst[m]);
          }
        }
    }
    if (has_terms && rnd > 0) e[1] = sub(cur, e[0]);  // (SKIP1 rounds; round 0 forms g(1) and checks the claim)
    Fr coeffs[4];
    interpolate4_host(e, coeffs);  // lagrange_interpolate of 4 points (src/sumcheck.rs:201-206)
    Fr g0 = horner_host(coeffs, 4, Fr::zero());
    Fr g1 = horner_host(coeffs, 4, Fr::one());
    if (add(g0, g1) != cur) {  // src/sumcheck.rs:80-84
      snprintf(lab, sizeof lab, "Round %u consistency check failed", rnd);
      throw Error(TNS_ERR_SUMCHECK, lab);
    }
    for (int x = 0; x < 4; x++) rounds[4 * rnd + x] = coeffs[x];
    snprintf(lab, sizeof lab, "sumcheck_round_%u", rnd);  // src/sumcheck.rs:90-96
    tr.append_label(lab);
    for (int x = 0; x < 4; x++) tr.append_fr(coeffs[x]);
    snprintf(lab, sizeof lab, "sumcheck_challenge_%u", rnd);
    Fr ch = tr.challenge(lab);
    if (challenges) challenges[rnd] = ch;
    cur = horner_host(coeffs, 4, ch);
    r_prev = ch;
  }
  // bind the last variable: final MLE values at (r_0..r_{nv-1}), in the caller's table order
  Fr vals[MAX_SC_TABLES];
  if (tail_rnd < nv) {
    // src: tables of n >> (tail_rnd - 1) entries; folds by the challenges of rounds
    // tail_rnd - 1 .. nv - 1 (the last one binds the final variable)
    const int m = (int)(nv - tail_rnd + 1);
    tail_ch[m - 1] = r_prev;
    Fr *d_ch = R.partials, *d_out = (Fr *)c->scratch[7].ensure(sizeof(Fr) * MAX_SC_TABLES);
    TNS_HIP(hipMemcpyAsync(d_ch, tail_ch, sizeof(Fr) * m, hipMemcpyHostToDevice, c->stream));
    ScTail tl{};
    for (int i = 0; i < k; i++) {  // src may still be the caller's table (tail from round 1); perm is identity here
      tl.a[i] = src[i];
      tl.b[i] = dst[i];
      tl.c[i] = src[i] == tables[R.perm[i]] ? bufC[R.perm[i]] : src[i];
    }
    TNS_PROF(c, "sumcheck_round", 96.0 * (double)(n >> (tail_rnd - 1)) * k);
    k_sc_fold_tail<<<1, 1024, 0, c->stream>>>(tl, k, m, d_ch, d_out);
    TNS_LAUNCH_CHECK();
    Fr kv[MAX_SC_TABLES];
    TNS_HIP(hipMemcpyAsync(kv, d_out, sizeof(Fr) * k, hipMemcpyDeviceToHost, c->stream));
    TNS_HIP(hipStreamSynchronize(c->stream));
    for (int m2 = 0; m2 < k; m2++) vals[R.perm[m2]] = kv[m2];
  } else if (k > 0) {
    ScTables tt{};
    for (int m2 = 0; m2 < k; m2++) tt.in[m2] = src[m2];
    const uint32_t seq = ++c->sc_seq;
    if (nv > 0) {  // (the challenge to device memory: k_sc_final reads it there)
      R.chal->r = r_prev;
      __atomic_store_n(&R.chal->flag, ++c->sc_chal_seq, __ATOMIC_RELEASE);
      k_sc_wait_r<<<1, 64, 0, c->stream>>>(R.chal_dev, c->sc_chal_seq, R.rd, R.res_dev);
      TNS_LAUNCH_CHECK();
    }
    k_sc_final<<<1, 64, 0, c->stream>>>(tt, k, R.rd, nv > 0, R.res_dev, seq);
    TNS_LAUNCH_CHECK();
    const ScResult &res = sc_wait(c, seq);
    for (int m2 = 0; m2 < k; m2++) vals[R.perm[m2]] = res.sums[m2];
  }
  for (int i = 0; i < k; i++) final_vals[i] = vals[i];
  *final_eval = eval_composition_host(vals, terms, n_terms);  // polynomial(&fixed_variables), :104
  // the last round's claim is g_{nv-1}(r_{nv-1}) = f(r): an honest prover's final value must equal
  // it; with g(1) taken from the claim (SKIP1) this is the check that catches a device miscompute
  if (has_terms && nv > 0 && *final_eval != cur)
    throw Error(TNS_ERR_SUMCHECK, "final evaluation does not match the last round's claim (device result inconsistent)");
  return TNS_OK;
}

}  // namespace tns
