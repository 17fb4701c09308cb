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

namespace tns {

constexpr int MAX_SC_TABLES = 4;
constexpr int MAX_SC_TERMS = 16;

struct ScTables {
  const Fr *in[MAX_SC_TABLES];
  Fr *out[MAX_SC_TABLES];
};
struct ScTerms {
  Fr coeff[MAX_SC_TERMS];
  int8_t tab[MAX_SC_TERMS][3];
  // coefficient kinds (set by sc_terms): 0 one, 1 minus one, 2 two, 3 any -- the round kernel
  // multiplies by a coefficient only for kind 3 (the Twist-shaped A V - O O V + 2 O: 3 products
  // per point instead of 6)
  int8_t kind[MAX_SC_TERMS];
  int n;
};

// the host side of ScTerms: tables checked against k, coefficient kinds classified
static ScTerms sc_terms(const SumcheckTerm *terms, int n_terms, int k) {
  if (n_terms > MAX_SC_TERMS) throw Error(TNS_ERR_INVALID_PARAMETERS, "at most 16 sum-check terms");
  ScTerms st{};
  st.n = n_terms;
  const Fr one = Fr::one(), two = add(one, one), minus_one = neg(one);
  for (int t = 0; t < n_terms; t++) {
    const Fr &c = terms[t].coeff;
    st.coeff[t] = c;
    st.kind[t] = c == one ? 0 : c == minus_one ? 1 : c == two ? 2 : 3;
    for (int j = 0; j < 3; j++) {
      const int ix = terms[t].tab[j];
      if (ix >= k) throw Error(TNS_ERR_INVALID_PARAMETERS, "term references a missing table");
      st.tab[t][j] = (int8_t)ix;
    }
  }
  return st;
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
// FOLD:   tables in[] have 4P entries; bind r into out[] (2P entries), then sum round values.
// !FOLD:  tables in[] have 2P entries (first round), just sum.
// Block partial sums (4 Fr: X = 0..3) -> partials[blockIdx.x * 4 + X].
// SKIP1: the sum at X = 1 is not formed (the host takes it as claim - g(0): from round 1 on the
// round polynomial's g(0) + g(1) equals the previous round's g(r) identically, src/sumcheck.rs:80-84)
template <bool FOLD, bool TERMS, bool SKIP1 = false>
__global__ void __launch_bounds__(256) k_sc_round(ScTables t, int k, ScTerms terms, size_t P, Fr r,
                                                  Fr *__restrict__ partials) {
  __shared__ Fr lds[4 * 16];
  Fr acc[4] = {Fr::zero(), Fr::zero(), Fr::zero(), Fr::zero()};
  for (size_t s = blockIdx.x * (size_t)blockDim.x + threadIdx.x; s < P;
       s += (size_t)gridDim.x * blockDim.x) {
    Fr f0[MAX_SC_TABLES], f1[MAX_SC_TABLES];
#pragma unroll
    for (int i = 0; i < MAX_SC_TABLES; i++) {
      if (i < k) {
        if (FOLD) {
          const Fr *p = t.in[i] + 4 * s;
          Fr x0 = p[0], x1 = p[1], x2 = p[2], x3 = p[3];
          f0[i] = add(x0, mul(r, sub(x1, x0)));
          f1[i] = add(x2, mul(r, sub(x3, x2)));
          t.out[i][2 * s] = f0[i];
          t.out[i][2 * s + 1] = f1[i];
        } else {
          f0[i] = t.in[i][2 * s];
          f1[i] = t.in[i][2 * s + 1];
        }
      }
    }
    if (TERMS) {
      // values at X = 0,1,2,3: f0, f1, f1 + d, f1 + 2d
      Fr d[MAX_SC_TABLES];
#pragma unroll
      for (int i = 0; i < MAX_SC_TABLES; i++)
        if (i < k) d[i] = sub(f1[i], f0[i]);
#pragma unroll  // (a runtime x put acc[] in scratch memory)
      for (int x = 0; x < 4; x++) {
        if (SKIP1 && x == 1) continue;
        Fr vx[MAX_SC_TABLES];
#pragma unroll
        for (int i = 0; i < MAX_SC_TABLES; i++) {
          if (i < k) {
            if (x == 0) vx[i] = f0[i];
            else if (x == 1) vx[i] = f1[i];
            else if (x == 2) vx[i] = add(f1[i], d[i]);
            else vx[i] = add(add(f1[i], d[i]), d[i]);
          }
        }
        Fr sum = Fr::zero();
        for (int tt = 0; tt < terms.n; tt++) {
          Fr p = Fr::one();
          bool first = true;
#pragma unroll
          for (int j = 0; j < 3; j++) {
            int ix = terms.tab[tt][j];
            if (ix >= 0) {
              Fr v = vx[0];
#pragma unroll
              for (int q = 1; q < MAX_SC_TABLES; q++)
                if (ix == q) v = vx[q];
              p = first ? v : mul(p, v);
              first = false;
            }
          }
          const int kind = terms.kind[tt];  // (uniform: the coefficient only where it is not +-1 or 2)
          if (kind == 1) p = neg(p);
          else if (kind == 2) p = add(p, p);
          else if (kind == 3) p = mul(terms.coeff[tt], p);
          sum = add(sum, p);
        }
        acc[x] = add(acc[x], sum);
      }
    }
  }
  if (TERMS) {
    block_sum_fr<4>(acc, lds);
    if (threadIdx.x == 0) {
#pragma unroll
      for (int x = 0; x < 4; x++) partials[blockIdx.x * 4 + x] = acc[x];
    }
  }
}

// Sum nb blocks' 4-vectors -> out[0..3]
__global__ void __launch_bounds__(256) k_sum_partials4(const Fr *__restrict__ partials, int nb,
                                                       Fr *__restrict__ out) {
  __shared__ Fr lds[4 * 16];
  Fr acc[4] = {Fr::zero(), Fr::zero(), Fr::zero(), Fr::zero()};
  for (int b = threadIdx.x; b < nb; b += blockDim.x)
    for (int x = 0; x < 4; x++) acc[x] = add(acc[x], partials[b * 4 + x]);
  block_sum_fr<4>(acc, lds);
  if (threadIdx.x == 0)
    for (int x = 0; x < 4; x++) out[x] = acc[x];
}

// Closure-free sum-check (no composition terms: every round polynomial is zero, so the
// challenges never wait for the device): the last m folds of the chain in one workgroup.
// Tables of 2^m entries in a[]; fold j binds ch[j] (LSB first, as k_sc_round) and ping-pongs
// a -> b -> a ...; out[i] = table i bound at all m challenges.  Replaces m - 1 small
// k_sc_round launches and the k final k_mle_fold launches (each ~20 us of launch gap).
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

static bool sc_fold3_on() {
  const char *f3 = getenv("TNS_SC_FOLD3");  // =0: one launch per round (A/B)
  return !(f3 && f3[0] == '0');
}

static unsigned sc_tail_round(unsigned nv) { return std::max(1u, nv + 1 - std::min(nv, SC_TAIL_LOG)); }

bool sumcheck_folds_take_flag_bytes(unsigned nv) { return sc_fold3_on() && sc_tail_round(nv) > 3; }

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
  // rounds 1 .. tail_rnd - 1 fold by r_{rnd-1} in k_sc_round; the rest (tables of <= 2^12) in
  // one k_sc_fold_tail workgroup, down to one value per table
  const unsigned tail_rnd = sc_tail_round(nv);
  Fr *src[MAX_SC_TABLES], *dst[MAX_SC_TABLES];
  for (int i = 0; i < k; i++) {
    src[i] = tables[i];
    dst[i] = bufB[i];
  }
  Fr ch[64];
  std::memcpy(ch, chal_pinned, sizeof(Fr) * std::min(nv, 64u));
  const bool fold3 = sc_fold3_on();
  bool first = true;
  for (unsigned rnd = 1; rnd < tail_rnd;) {
    ScTables tt{};
    for (int i = 0; i < k; i++) {
      tt.in[i] = src[i];
      tt.out[i] = dst[i];
    }
    if (fold3 && rnd + 2 < tail_rnd) {  // rounds rnd .. rnd + 2 in one pass
      const size_t P = n >> (rnd + 2);
      TNS_PROF_ON(c, st, "sumcheck_round", 288.0 * (double)P * k);
      k_sc_fold3<<<grid_for(P, 256, 4096), 256, 0, st>>>(tt, k, P, ch[rnd - 1], ch[rnd], ch[rnd + 1],
                                                          first ? flags : nullptr, n_flags);
      TNS_LAUNCH_CHECK();
      rnd += 3;
    } else {
      const size_t P = n >> (rnd + 1);
      TNS_PROF_ON(c, st, "sumcheck_round", 192.0 * (double)P * k);
      k_sc_round<true, false><<<grid_for(P, 256, 2048), 256, 0, st>>>(tt, k, ScTerms{}, P, ch[rnd - 1], nullptr);
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

// sum over {0,1}^nv of the composition (the honest prover's claimed sum): round 0's sums at
// X = 0 and X = 1 of the fused round kernel, added
Fr composition_sum_dev(Ctx *c, Fr *const *tables, int k, unsigned nv, const SumcheckTerm *terms, int n_terms) {
  if (k < 1 || k > MAX_SC_TABLES) throw Error(TNS_ERR_INVALID_PARAMETERS, "1 to 4 sum-check tables");
  const ScTerms st = sc_terms(terms, n_terms, k);
  if (nv == 0) {
    Fr v[MAX_SC_TABLES];
    for (int i = 0; i < k; i++) TNS_HIP(hipMemcpyAsync(&v[i], tables[i], sizeof(Fr), hipMemcpyDeviceToHost, c->stream));
    TNS_HIP(hipStreamSynchronize(c->stream));
    return eval_composition_host(v, terms, n_terms);
  }
  const size_t P = (size_t)1 << (nv - 1);
  const unsigned g = grid_for(P, 256, 2048);
  Fr *partials = (Fr *)c->scratch[6].ensure(sizeof(Fr) * std::max<size_t>(4 * (size_t)g, 64));
  Fr *sums_dev = (Fr *)c->scratch[7].ensure(sizeof(Fr) * 4);
  ScTables tt{};
  for (int i = 0; i < k; i++) tt.in[i] = tables[i];
  k_sc_round<false, true><<<g, 256, 0, c->stream>>>(tt, k, st, P, Fr::zero(), partials);
  TNS_LAUNCH_CHECK();
  k_sum_partials4<<<1, 256, 0, c->stream>>>(partials, (int)g, sums_dev);
  TNS_LAUNCH_CHECK();
  Fr e[4];
  TNS_HIP(hipMemcpyAsync(e, sums_dev, sizeof e, hipMemcpyDeviceToHost, c->stream));
  TNS_HIP(hipStreamSynchronize(c->stream));
  return add(e[0], e[1]);
}

// SumCheck::prove (src/sumcheck.rs:56-110) for an MLE composition.
// tables: k device arrays of 2^nv Fr (read only).  Host transcript drives challenges.
int sumcheck_prove_dev(Ctx *c, Fr *const *tables, int k, unsigned nv, const Fr &claimed,
                       const SumcheckTerm *terms, int n_terms, HostTranscript &tr, Fr *rounds,
                       Fr *challenges, Fr *final_vals, Fr *final_eval) {
  if (k < 0 || k > MAX_SC_TABLES) throw Error(TNS_ERR_INVALID_PARAMETERS, "at most 4 sum-check tables");
  const ScTerms st = sc_terms(terms, n_terms, k);
  const bool has_terms = n_terms > 0;
  const size_t n = (size_t)1 << nv;
  // ping-pong: round r (r >= 1) reads src (2^(nv-r+1)) and writes dst (2^(nv-r)); round 1
  // reads the caller's tables, later rounds alternate between bufB and bufC, so the input
  // tables are left intact (Twist / Shout open the same evaluation vectors afterwards).
  Fr *bufB[MAX_SC_TABLES], *bufC[MAX_SC_TABLES];
  for (int i = 0; i < k; i++) {
    bufB[i] = (Fr *)c->scratch[2 + i].ensure(sizeof(Fr) * (n / 2 + 1));
    bufC[i] = (Fr *)c->sc_pong[i].ensure(sizeof(Fr) * (n / 4 + 1));
  }
  const int nblk = (int)grid_for(n / 2 + 1, 256, 2048);
  Fr *partials = (Fr *)c->scratch[6].ensure(sizeof(Fr) * std::max<size_t>(4 * (size_t)nblk, 64));
  Fr *sums_dev = (Fr *)c->scratch[7].ensure(sizeof(Fr) * 4);

  Fr cur = claimed;
  Fr *src[MAX_SC_TABLES], *dst[MAX_SC_TABLES];
  for (int i = 0; i < k; i++) {
    src[i] = tables[i];
    dst[i] = bufB[i];
  }
  Fr r_prev = Fr::zero();
  char lab[64];
  // closure-free chains hand their last folds to k_sc_fold_tail: from round `tail_rnd` on
  // (input tables of n >> (tail_rnd - 1) <= 2^SC_TAIL_LOG entries) only the transcript runs
  const unsigned tail_rnd =
      (c->sc_tail && !has_terms && k > 0 && nv >= 2) ? std::max(1u, nv + 1 - std::min(nv, SC_TAIL_LOG)) : nv + 1;
  Fr tail_ch[64];
  for (unsigned rnd = 0; rnd < nv; rnd++) {
    const size_t P = n >> (rnd + 1);  // output pairs of this round
    const unsigned g = grid_for(P, 256, 2048);
    if (rnd >= tail_rnd) {
      tail_ch[rnd - tail_rnd] = r_prev;  // this round's fold runs in k_sc_fold_tail
    } else {
      ScTables tt{};
      for (int i = 0; i < k; i++) {
        tt.in[i] = src[i];
        tt.out[i] = dst[i];
      }
      TNS_PROF(c, "sumcheck_round", (rnd == 0 ? 64.0 : 192.0) * (double)P * k);
      if (rnd == 0) {
        if (has_terms) k_sc_round<false, true><<<g, 256, 0, c->stream>>>(tt, k, st, P, r_prev, partials);
      } else {
        if (has_terms)
          k_sc_round<true, true, true><<<g, 256, 0, c->stream>>>(tt, k, st, P, r_prev, partials);
        else
          k_sc_round<true, false><<<g, 256, 0, c->stream>>>(tt, k, st, P, r_prev, partials);
        // src now holds the freshly folded 2P-entry tables
        for (int i = 0; i < k; i++) {
          if (rnd == 1) {
            src[i] = bufB[i];
            dst[i] = bufC[i];
          } else {
            std::swap(src[i], dst[i]);
          }
        }
      }
      TNS_LAUNCH_CHECK();
    }
    Fr e[4] = {Fr::zero(), Fr::zero(), Fr::zero(), Fr::zero()};
    if (has_terms) {
      k_sum_partials4<<<1, 256, 0, c->stream>>>(partials, (int)g, sums_dev);
      TNS_LAUNCH_CHECK();
      TNS_HIP(hipMemcpyAsync(e, sums_dev, sizeof e, hipMemcpyDeviceToHost, c->stream));
      TNS_HIP(hipStreamSynchronize(c->stream));
      if (rnd > 0) e[1] = sub(cur, e[0]);  // (SKIP1 rounds; round 0 forms g(1) and checks the claim)
    }
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
  // bind the last variable: final MLE values at (r_0..r_{nv-1})
  Fr vals[MAX_SC_TABLES];
  if (tail_rnd < nv) {
    // src: tables of n >> (tail_rnd - 1) entries; folds by the challenges of rounds
    // tail_rnd - 1 .. nv - 1 (the last one binds the final variable)
    const int m = (int)(nv - tail_rnd + 1);
    tail_ch[m - 1] = r_prev;
    Fr *d_ch = partials, *d_out = sums_dev;
    TNS_HIP(hipMemcpyAsync(d_ch, tail_ch, sizeof(Fr) * m, hipMemcpyHostToDevice, c->stream));
    ScTail tl{};
    for (int i = 0; i < k; i++) {  // src may still be the caller's table (tail from round 1)
      tl.a[i] = src[i];
      tl.b[i] = dst[i];
      tl.c[i] = src[i] == tables[i] ? bufC[i] : src[i];
    }
    TNS_PROF(c, "sumcheck_round", 96.0 * (double)(n >> (tail_rnd - 1)) * k);
    k_sc_fold_tail<<<1, 1024, 0, c->stream>>>(tl, k, m, d_ch, d_out);
    TNS_LAUNCH_CHECK();
    TNS_HIP(hipMemcpyAsync(vals, d_out, sizeof(Fr) * k, hipMemcpyDeviceToHost, c->stream));
  } else {
    for (int i = 0; i < k; i++) {
      if (nv == 0) {
        TNS_HIP(hipMemcpyAsync(&vals[i], src[i], sizeof(Fr), hipMemcpyDeviceToHost, c->stream));
      } else {
        mle_fold_dev(c, src[i], dst[i], 1, r_prev);
        TNS_HIP(hipMemcpyAsync(&vals[i], dst[i], sizeof(Fr), hipMemcpyDeviceToHost, c->stream));
      }
    }
  }
  TNS_HIP(hipStreamSynchronize(c->stream));
  for (int i = 0; i < k; i++) final_vals[i] = vals[i];
  *final_eval = eval_composition_host(vals, terms, n_terms);  // polynomial(&fixed_variables), :104
  return TNS_OK;
}

}  // namespace tns
