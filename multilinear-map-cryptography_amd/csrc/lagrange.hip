// lagrange.hip -- KZG commit/open directly on evaluations over the nodes {0..N-1}.
//
// The reference commits to vector_to_polynomial(v) (src/polynomials.rs:248-262): the
// coefficients of the interpolant of v on the nodes 0..N-1, then C = sum_i c_i tau^i G
// (src/commitments.rs:162-180), and opens with P(z) and the commitment to
// (P(x) - P(z)) / (x - z) (src/commitments.rs:182-199).  Both group elements are
// values of polynomials at tau, so with the Lagrange basis of those nodes
//     L_j(tau) = ell(tau) * w_j / (tau - j),  ell(x) = prod_k (x - k),
//     w_j = 1 / prod_{k != j} (j - k) = (-1)^(N-1-j) / (j! (N-1-j)!)
// they are the same points computed without the coefficient form:
//     commit:  C  = sum_j v_j * [L_j(tau)] G
//     open:    P(z) = ell(z) * sum_j w_j v_j / (z - j)        (barycentric form)
//              pi = sum_j q_j [L_j(tau)] G,  q_j = (P(z) - v_j) / (z - j)
// (q has degree N - 2, so its values on the N nodes determine it exactly).  The basis
// [L_j(tau)] G is derived once per N from the setup's tau -- the same trusted-setup
// output as the powers g1_powers, like the Lagrange-form SRS of production KZG
// ceremonies -- and cached with the SRS.  Each proof is then O(N) field work plus the
// MSMs; the interpolation (interp.hip) stays the path for SRSs without tau and for the
// probability-2^-230 case of a challenge that lands on a node.
//
// One O(N) building block serves both: inverses of (x - j) for all nodes by a batch
// inversion whose per-thread chains stride the array (coalesced), with ell(x) as the
// product of the chain products.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <tuple>
#include <vector>

#include "common.hpp"
#include "hostfield.hpp"

namespace tns {

constexpr unsigned NODE_THREADS = 512 * 256;  // batch-inversion chains (one Fermat inverse each)

// chain t: elements i = t + k*T.  pre[i] = prod of earlier (x - i') of the chain; cp[t] = chain
// product.  Node `skip` (x itself, when opening at a node) contributes the factor 1.
__global__ void __launch_bounds__(256) k_node_chain(Fr x, size_t n, size_t T, Fr Tm, size_t skip,
                                                    Fr *__restrict__ pre, Fr *__restrict__ cp) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (t >= T) return;
  Fr d = sub(x, from_u64<FrCfg>((uint64_t)t));  // x - i, stepping by -T
  Fr acc = Fr::one();
  for (size_t i = t; i < n; i += T) {
    pre[i] = acc;
    if (i != skip) acc = mul(acc, d);
    d = sub(d, Tm);
  }
  cp[t] = acc;
}

// icp[t] = 1 / cp[t] for t < T by one batch inversion per block of 256 chains (prefix and suffix
// products in LDS, one Fermat inverse per block instead of one per chain: those were about a
// third of k_node_finish2's multiplies).  A zero chain product gets 0 and leaves its block's
// other inverses intact.  scale multiplies every inverse (the raw 1 = R^-1: canonical outputs,
// see lagrange_open_partial2_dev).  blockDim.x == 256.
__global__ void __launch_bounds__(256) k_chain_inv(const Fr *__restrict__ cp, size_t T, Fr *__restrict__ icp,
                                                   Fr scale) {
  __shared__ Fr sh[256];
  __shared__ Fr inv_total;
  const int tid = threadIdx.x;
  const size_t t = blockIdx.x * (size_t)blockDim.x + tid;
  Fr a = t < T ? cp[t] : Fr::one();
  const bool zero = a.is_zero();
  if (zero) a = Fr::one();
  Fr lo = a, hi = a;  // inclusive prefix / suffix products over the block
  for (int off = 1; off < 256; off <<= 1) {
    sh[tid] = lo;
    __syncthreads();
    const Fr o = tid >= off ? sh[tid - off] : Fr::one();
    __syncthreads();
    lo = mul(o, lo);
  }
  for (int off = 1; off < 256; off <<= 1) {
    sh[tid] = hi;
    __syncthreads();
    const Fr o = tid + off < 256 ? sh[tid + off] : Fr::one();
    __syncthreads();
    hi = mul(hi, o);
  }
  // hi of thread 0 = the block's product; its inverse is the kernel's latency: the binary extended
  // Euclid (TNS_CHAIN_INV_FERMAT=1 build: the Fermat chain)
#if defined(TNS_CHAIN_INV_FERMAT)
  if (tid == 0) inv_total = mul(inv(hi), scale);
#else
  if (tid == 0) inv_total = mul(inv_binary_dev(hi), scale);
#endif
  sh[tid] = lo;
  __syncthreads();
  const Fr before = tid ? sh[tid - 1] : Fr::one();  // prod over s < t
  __syncthreads();
  sh[tid] = hi;
  __syncthreads();
  const Fr after = tid < 255 ? sh[tid + 1] : Fr::one();  // prod over s > t
  if (t < T) icp[t] = zero ? Fr::zero() : mul(mul(before, after), inv_total);
}

// The same batch inversion with ONE inverse for the whole grid, taken on the host: a single-lane
// binary Euclid per block (k_chain_inv) is ~0.15-0.2 ms of dependent 256-bit steps on the
// barycentric pass's critical path, the host's 4 x u64 inverse ~20 us.
// (1) per block of 256 chains: icp[t] = the product of the block's OTHER chains, tot[b] = the block's
//     product (zero chains count as one and are flagged: their inverse is 0);
__global__ void __launch_bounds__(256) k_chain_local(const Fr *__restrict__ cp, size_t T, Fr *__restrict__ icp,
                                                     Fr *__restrict__ tot) {
  __shared__ Fr sh[256];
  const int tid = threadIdx.x;
  const size_t t = blockIdx.x * (size_t)blockDim.x + tid;
  Fr a = t < T ? cp[t] : Fr::one();
  const bool zero = a.is_zero();
  if (zero) a = Fr::one();
  Fr lo = a, hi = a;  // inclusive prefix / suffix products over the block
  for (int off = 1; off < 256; off <<= 1) {
    sh[tid] = lo;
    __syncthreads();
    const Fr o = tid >= off ? sh[tid - off] : Fr::one();
    __syncthreads();
    lo = mul(o, lo);
  }
  for (int off = 1; off < 256; off <<= 1) {
    sh[tid] = hi;
    __syncthreads();
    const Fr o = tid + off < 256 ? sh[tid + off] : Fr::one();
    __syncthreads();
    hi = mul(hi, o);
  }
  if (tid == 0) tot[blockIdx.x] = hi;
  sh[tid] = lo;
  __syncthreads();
  const Fr before = tid ? sh[tid - 1] : Fr::one();
  __syncthreads();
  sh[tid] = hi;
  __syncthreads();
  const Fr after = tid < 255 ? sh[tid + 1] : Fr::one();
  if (t < T) icp[t] = zero ? Fr::zero() : mul(before, after);
}

// (2) one block over the nb <= 1024 block products: oth[b] = the product of the OTHER blocks, and the
//     grand product to the host (mapped memory, then the flag)
__global__ void __launch_bounds__(256) k_chain_totals(const Fr *__restrict__ tot, int nb, Fr *__restrict__ oth,
                                                      Fr *pub, uint32_t *flag, uint32_t seq) {
  __shared__ Fr sh[256];
  constexpr int PER = 4;  // blocks per thread (nb <= 1024)
  const int tid = threadIdx.x;
  Fr v[PER], lo = Fr::one();
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const int b = tid * PER + k;
    v[k] = b < nb ? tot[b] : Fr::one();
    lo = mul(lo, v[k]);
  }
  Fr hi = lo;
  const Fr mine = lo;
  for (int off = 1; off < 256; off <<= 1) {
    sh[tid] = lo;
    __syncthreads();
    const Fr o = tid >= off ? sh[tid - off] : Fr::one();
    __syncthreads();
    lo = mul(o, lo);
  }
  for (int off = 1; off < 256; off <<= 1) {
    sh[tid] = hi;
    __syncthreads();
    const Fr o = tid + off < 256 ? sh[tid + off] : Fr::one();
    __syncthreads();
    hi = mul(hi, o);
  }
  sh[tid] = lo;
  __syncthreads();
  Fr before = tid ? sh[tid - 1] : Fr::one();  // blocks of the threads before this one
  __syncthreads();
  sh[tid] = hi;
  __syncthreads();
  const Fr after = tid < 255 ? sh[tid + 1] : Fr::one();
  (void)mine;
  // inside the thread: prefix and suffix over its PER blocks
  Fr suf[PER];
  suf[PER - 1] = Fr::one();
#pragma unroll
  for (int k = PER - 2; k >= 0; k--) suf[k] = mul(suf[k + 1], v[k + 1]);
#pragma unroll
  for (int k = 0; k < PER; k++) {
    const int b = tid * PER + k;
    if (b < nb) oth[b] = mul(mul(before, suf[k]), after);
    before = mul(before, v[k]);
  }
  if (tid == 0) {
    *pub = hi;  // thread 0's suffix = every block's product
    __threadfence_system();
    __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// (3) icp[t] *= oth[block of t] * inv_all (the host's inverse of the grand product, times scale)
__global__ void __launch_bounds__(256) k_chain_apply(Fr *__restrict__ icp, size_t T, const Fr *__restrict__ oth,
                                                     Fr inv_all) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (t >= T) return;
  const Fr o = mul(oth[blockIdx.x], inv_all);
  icp[t] = mul(icp[t], o);  // (a flagged zero chain stays 0)
}

// out[blockIdx.x] = prod of in[i] over the block's grid-stride share (one level of a product tree)
__global__ void __launch_bounds__(256) k_prod_reduce(const Fr *__restrict__ in, size_t n, Fr *__restrict__ out) {
  __shared__ Fr lds[256];
  Fr acc = Fr::one();
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc = mul(acc, in[i]);
  lds[threadIdx.x] = acc;
  __syncthreads();
  for (unsigned s = blockDim.x / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) lds[threadIdx.x] = mul(lds[threadIdx.x], lds[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = lds[0];
}

// *out = prod_i in[i]: a 256-block level into tmp[0..256), then one block
static void prod_reduce(hipStream_t st, const Fr *in, size_t n, Fr *tmp, Fr *out) {
  if (n > 4096) {
    k_prod_reduce<<<256, 256, 0, st>>>(in, n, tmp);
    TNS_LAUNCH_CHECK();
    in = tmp;
    n = 256;
  }
  k_prod_reduce<<<1, 256, 0, st>>>(in, n, out);
  TNS_LAUNCH_CHECK();
}

// Backward sweep of chain t: inv_i = 1/(x - i) from pre[i] and the chain inverse.
//   BASIS: out[i] = canonical(ell * w_i * inv_i)                  (Lagrange scalars L_i(x))
//   OPEN:  out[i] = inv_i, sp[t] = sum_chain w_i (y_i - yoff) inv_i (barycentric partial sum)
// The punctured node `skip` (opening at a node) gets inv 0 and no sum term.
template <bool BASIS>
// (pre and out may alias: each element's pre is read before its output is written)
__global__ void __launch_bounds__(256) k_node_finish(Fr x, size_t n, size_t T, Fr Tm, size_t skip, Fr yoff,
                                                     const Fr *pre, const Fr *__restrict__ cp, bool inverted,
                                                     const Fr *__restrict__ w, const Fr *__restrict__ y,
                                                     const Fr *__restrict__ ell, Fr *out, Fr *__restrict__ sp) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (t >= T) return;
  if (t >= n) {
    if (!BASIS) sp[t] = Fr::zero();
    return;
  }
  const size_t cnt = (n - 1 - t) / T;  // index of the chain's last element
  size_t i = t + cnt * T;
  Fr d = sub(x, from_u64<FrCfg>((uint64_t)i));
  Fr iv = inverted ? cp[t] : inv(cp[t]);  // cp: the chain inverses (k_chain_inv) or products
  Fr s = Fr::zero();
  const Fr L = BASIS ? ell[0] : Fr::one();
  for (;;) {
    const bool hole = i == skip;
    const Fr inv_i = hole ? Fr::zero() : mul(iv, pre[i]);
    if (!hole) iv = mul(iv, d);
    if (BASIS) {
      out[i] = from_mont(mul(mul(L, w[i]), inv_i));
    } else {
      out[i] = inv_i;
      s = add(s, mul(mul(w[i], sub(y[i], yoff)), inv_i));
    }
    if (i < T) break;
    i -= T;
    d = add(d, Tm);
  }
  if (!BASIS) sp[t] = s;
}

// k_node_finish<false> for two vectors on the same nodes: the inverses are shared.
//   inv[i] = inv_i;  sp[t] = sum_chain w_i y0_i inv_i,  sp[T + t] = sum_chain w_i y1_i inv_i
// scale: as k_chain_inv's (applied here when the chain products come uninverted)
__global__ void __launch_bounds__(256) k_node_finish2(Fr x, size_t n, size_t T, Fr Tm, const Fr *pre,
                                                      const Fr *__restrict__ cp, bool inverted, Fr scale,
                                                      const Fr *__restrict__ w, const Fr *__restrict__ y0,
                                                      const Fr *__restrict__ y1, Fr *invs, Fr *__restrict__ sp) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (t >= T) return;
  if (t >= n) {
    sp[t] = sp[T + t] = Fr::zero();
    return;
  }
  const size_t cnt = (n - 1 - t) / T;
  size_t i = t + cnt * T;
  Fr d = sub(x, from_u64<FrCfg>((uint64_t)i));
  Fr iv = inverted ? cp[t] : mul(inv(cp[t]), scale);  // cp: the chain inverses (k_chain_inv) or products
  Fr s0 = Fr::zero(), s1 = Fr::zero();
  for (;;) {
    const Fr inv_i = mul(iv, pre[i]);
    iv = mul(iv, d);
    invs[i] = inv_i;
    const Fr wi = mul(w[i], inv_i);
    s0 = add(s0, mul(wi, y0[i]));
    s1 = add(s1, mul(wi, y1[i]));
    if (i < T) break;
    i -= T;
    d = add(d, Tm);
  }
  sp[t] = s0;
  sp[T + t] = s1;
}

// q0_i = (v0 - y0_i) inv_i, q1_i = (v1 - y1_i) inv_i; q1 may alias inv
__global__ void __launch_bounds__(256) k_node_quotient2(const Fr *__restrict__ y0, const Fr *__restrict__ y1, Fr v0,
                                                        Fr v1, size_t n, const Fr *invs, Fr *__restrict__ q0, Fr *q1) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const Fr iv = invs[i];
    q0[i] = mul(sub(v0, y0[i]), iv);
    q1[i] = mul(sub(v1, y1[i]), iv);
  }
}

// k_node_quotient2 producing what the two opening MSMs consume: the CANONICAL quotient values
// (the bucket sort reads digits of canonical scalars) and each vector's largest bit length
// (the MSM's window plan) -- msm.hip's k_scalar_bits pass over q0 / q1 is folded in here.
// CI: the inverses are stored canonical (raw integers, i.e. the Montgomery forms of inv / R), so
// the Montgomery product (v - y) * inv already IS the canonical quotient -- no reduction pass.
template <bool CI>
__global__ void __launch_bounds__(256) k_node_quotient2_canon(const Fr *__restrict__ y0, const Fr *__restrict__ y1,
                                                              Fr v0, Fr v1, size_t n, const Fr *invs,
                                                              Fr *__restrict__ q0, Fr *q1, unsigned *__restrict__ bits) {
  unsigned b0 = 0, b1 = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const Fr iv = invs[i];
    Fr c0 = mul(sub(v0, y0[i]), iv), c1 = mul(sub(v1, y1[i]), iv);
    if (!CI) {
      c0 = from_mont(c0);
      c1 = from_mont(c1);
    }
    q0[i] = c0;
    q1[i] = c1;
    b0 = max(b0, fr_bit_length(c0));
    b1 = max(b1, fr_bit_length(c1));
  }
  block_atomic_max2(b0, b1, bits, bits + 1);
}

// q_i = (v - y_i) * inv_i, in place over inv
__global__ void __launch_bounds__(256) k_node_quotient(const Fr *__restrict__ y, Fr v, size_t n, Fr *__restrict__ q) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    q[i] = mul(sub(v, y[i]), q[i]);
}

// w[i] = w_j for j = first + i:  w_j = (-1)^(N-1-j) / (j! (N-1-j)!)
__global__ void __launch_bounds__(256) k_bary_weights(const Fr *__restrict__ ifact, size_t N, size_t first,
                                                      size_t cnt, Fr *__restrict__ w) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < cnt; i += (size_t)gridDim.x * blockDim.x) {
    const size_t j = first + i;
    Fr x = mul(ifact[j], ifact[N - 1 - j]);
    w[i] = ((N - 1 - j) & 1) ? neg(x) : x;
  }
}

// cp[t] = prod over the chain t of (x - i), i = t, t + T, ... < n (no per-node output)
__global__ void __launch_bounds__(256) k_node_prod(Fr x, size_t n, size_t T, Fr Tm, Fr *__restrict__ cp) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (t >= T) return;
  Fr d = sub(x, from_u64<FrCfg>((uint64_t)t));
  Fr acc = Fr::one();
  for (size_t i = t; i < n; i += T) {
    acc = mul(acc, d);
    d = sub(d, Tm);
  }
  cp[t] = acc;
}

// out[0] = sum_i in[i] (one block)
__global__ void __launch_bounds__(1024) k_sum_reduce(const Fr *__restrict__ in, size_t n, Fr *__restrict__ out) {
  __shared__ Fr lds[1024];
  Fr acc = Fr::zero();
  for (size_t i = threadIdx.x; i < n; i += blockDim.x) acc = add(acc, in[i]);
  lds[threadIdx.x] = acc;
  __syncthreads();
  for (unsigned s = blockDim.x / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) lds[threadIdx.x] = add(lds[threadIdx.x], lds[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = lds[0];
}

// barycentric weights of the nodes [first, first + cnt) of {0..N-1} (cached per slice)
static const Fr *bary_weights(Ctx *c, size_t N, size_t first, size_t cnt) {
  const auto key = std::make_tuple(N, first, cnt);
  auto it = c->bary_w.find(key);
  if (it != c->bary_w.end()) return it->second->as<Fr>();
  DevBuf fact, ifact;
  Fr *f = (Fr *)fact.ensure(sizeof(Fr) * N), *fi = (Fr *)ifact.ensure(sizeof(Fr) * N);
  factorial_tables_dev(c, N, f, fi);
  DevBuf *b = new DevBuf();
  Fr *w = (Fr *)b->ensure(sizeof(Fr) * cnt);
  k_bary_weights<<<grid_for(cnt, 256), 256, 0, c->stream>>>(fi, N, first, cnt, w);
  TNS_LAUNCH_CHECK();
  TNS_HIP(hipStreamSynchronize(c->stream));  // fact/ifact die here
  c->bary_w[key] = b;
  return w;
}

const Fr *bary_weights_dev(Ctx *c, size_t N, size_t first, size_t cnt) { return bary_weights(c, N, first, cnt); }

bool fr_is_node(const Fr &x, size_t N) {
  Fr k = from_mont(x);
  for (int i = 2; i < 8; i++)
    if (k.v[i]) return false;
  const uint64_t v = (uint64_t)k.v[0] | ((uint64_t)k.v[1] << 32);
  return v < N;
}

// (2^16 / 2^17 / 2^18 chains: 1.92 / 1.58 / 1.64 ms of barycentric pass at C4)
static size_t chain_count(size_t n) { return n < (size_t)NODE_THREADS ? n : (size_t)NODE_THREADS; }

struct NodeSweep {
  size_t T;
  Fr Tm;
  Fr *cp, *sp, *dev;  // chain products, partial sums, device scalars
  Fr *icp;            // what the finish kernels read: the chain inverses, or cp (inverted = false)
  bool inverted;
};

// chains over the local nodes i < n of x' = x - first (so x' - i = x - j); dev[0] = prod
static NodeSweep node_sweep_begin(Ctx *c, const Fr &xs, size_t n, Fr *pre, size_t skip = SIZE_MAX,
                                   const Fr &scale = Fr::one(), const std::function<void()> &queued = nullptr) {
  NodeSweep s;
  s.T = chain_count(n);
  s.Tm = from_u64<FrCfg>((uint64_t)s.T);
  Fr *ws = (Fr *)c->scratch[5].ensure(sizeof(Fr) * (4 * s.T + 4 + 256));
  s.cp = ws;
  s.sp = ws + s.T;  // 2T: room for two vectors' partial sums
  s.dev = ws + 3 * s.T;
  k_node_chain<<<grid_for(s.T, 256, 1u << 30), 256, 0, c->stream>>>(xs, n, s.T, s.Tm, skip, pre, s.cp);
  TNS_LAUNCH_CHECK();
  prod_reduce(c->stream, s.cp, s.T, s.dev + 4, s.dev);
  // the chain products' inverses: one batch inversion over all chains, its single inverse on the host
  s.inverted = true;
  s.icp = s.dev + 4 + 256;
  const unsigned nb = grid_for(s.T, 256, 1u << 30);
  Fr *tot = (Fr *)c->scratch[6].ensure(sizeof(Fr) * 2 * nb), *oth = tot + nb;
  if (nb > 1024) {  // (more than 2^18 chains: one inverse per block, on the device)
    k_chain_inv<<<nb, 256, 0, c->stream>>>(s.cp, s.T, s.icp, scale);
    TNS_LAUNCH_CHECK();
    if (queued) queued();
    return s;
  }
  k_chain_local<<<nb, 256, 0, c->stream>>>(s.cp, s.T, s.icp, tot);
  TNS_LAUNCH_CHECK();
  char *m = (char *)c->inv_mapped.ensure(64 + sizeof(Fr));
  const uint32_t seq = ++c->inv_seq;
  k_chain_totals<<<1, 256, 0, c->stream>>>(tot, (int)nb, oth, (Fr *)((char *)c->inv_mapped.dev + 64),
                                           (uint32_t *)c->inv_mapped.dev, seq);
  TNS_LAUNCH_CHECK();
  if (queued) queued();  // (under the chain kernels, ~0.6 ms at C4)
  const volatile uint32_t *flag = (const volatile uint32_t *)m;
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned spin = 1; __atomic_load_n((const uint32_t *)flag, __ATOMIC_ACQUIRE) != seq; spin++)
    if ((spin & 4095) == 0) {  // a faulted stream reports here instead of leaving the flag unset
      const hipError_t e = hipStreamQuery(c->stream);
      if (e != hipSuccess && e != hipErrorNotReady) TNS_HIP(e);
      if (e == hipSuccess && __atomic_load_n((const uint32_t *)flag, __ATOMIC_ACQUIRE) != seq)
        throw Error(TNS_ERR_DEVICE, "batch inversion: stream idle without its grand product");
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > 120.0)
        throw Error(TNS_ERR_DEVICE, "batch inversion: grand product did not arrive within 120 s");
    }
  Fr all;
  std::memcpy(&all, m + 64, sizeof(Fr));
  const Fr inv_all = mul(h_inv(HFr::of(all)).fp(), scale);  // (all != 0: zero chains count as one)
  k_chain_apply<<<nb, 256, 0, c->stream>>>(s.icp, s.T, oth, inv_all);
  TNS_LAUNCH_CHECK();
  return s;
}

static Fr fr_shift(const Fr &x, size_t first) { return sub(x, from_u64<FrCfg>((uint64_t)first)); }

const LagrangeBasis *lagrange_basis_dev(Ctx *c, const Srs &srs, size_t N, size_t first, size_t cnt) {
  if (!c->lagrange_commit || N == 0) return nullptr;
  if (first + cnt > N || cnt == 0) throw Error(TNS_ERR_INVALID_PARAMETERS, "node slice outside 0..N-1");
  const auto key = std::make_tuple(N, first, cnt);
  auto it = srs.lagrange.find(key);
  if (it != srs.lagrange.end()) return it->second;  // also a basis built from g1_powers alone (tfree.hip)
  if (!srs.has_tau || fr_is_node(srs.tau, N)) return nullptr;
  const Fr *w = bary_weights(c, N, first, cnt);
  // ell(tau) over all N nodes
  DevBuf ellb;
  const size_t TG = chain_count(N);
  Fr *ecp = (Fr *)ellb.ensure(sizeof(Fr) * (TG + 1));
  k_node_prod<<<grid_for(TG, 256, 1u << 30), 256, 0, c->stream>>>(srs.tau, N, TG, from_u64<FrCfg>((uint64_t)TG),
                                                                   ecp);
  TNS_LAUNCH_CHECK();
  DevBuf tmpb;
  prod_reduce(c->stream, ecp, TG, (Fr *)tmpb.ensure(sizeof(Fr) * 256), ecp + TG);
  DevBuf scal;
  Fr *sc = (Fr *)scal.ensure(sizeof(Fr) * cnt);  // pre, then canonical L_j(tau) in place
  const Fr xs = fr_shift(srs.tau, first);
  NodeSweep s = node_sweep_begin(c, xs, cnt, sc);
  k_node_finish<true><<<grid_for(s.T, 256, 1u << 30), 256, 0, c->stream>>>(xs, cnt, s.T, s.Tm, SIZE_MAX, Fr::zero(),
                                                                           sc, s.icp, s.inverted, w, nullptr, ecp + TG, sc,
                                                                           nullptr);
  TNS_LAUNCH_CHECK();
  LagrangeBasis *b = new LagrangeBasis();
  try {
    G1Affine *pts = (G1Affine *)b->points.ensure(sizeof(G1Affine) * cnt);
    fixed_base_mul_dev(c, sc, cnt, pts);  // synchronises
    if (cnt >= ((size_t)1 << 12)) b->fb = fixed_base_try_build(c, pts, cnt);
  } catch (...) {
    delete b;
    throw;
  }
  srs.lagrange[key] = b;
  return b;
}

void lagrange_open_partial_dev(Ctx *c, const Fr *y, size_t N, size_t first, size_t cnt, const Fr &z, Fr *inv,
                               Fr *ell_part, Fr *sum_part) {
  TNS_PROF(c, "open_scan", 32.0 * 4 * cnt);  // pre write/read, inv write, y, w
  const Fr *w = bary_weights(c, N, first, cnt);
  const Fr xs = fr_shift(z, first);
  NodeSweep s = node_sweep_begin(c, xs, cnt, inv);
  k_node_finish<false><<<grid_for(s.T, 256, 1u << 30), 256, 0, c->stream>>>(xs, cnt, s.T, s.Tm, SIZE_MAX, Fr::zero(),
                                                                            inv, s.icp, s.inverted, w, y, nullptr, inv,
                                                                            s.sp);
  TNS_LAUNCH_CHECK();
  k_sum_reduce<<<1, 1024, 0, c->stream>>>(s.sp, s.T, s.dev + 1);
  TNS_LAUNCH_CHECK();
  Fr h[2];
  TNS_HIP(hipMemcpyAsync(h, s.dev, sizeof h, hipMemcpyDeviceToHost, c->stream));
  TNS_HIP(hipStreamSynchronize(c->stream));
  *ell_part = h[0];
  *sum_part = h[1];
}

// Opening at the node j0 (KZGVectorCommitment::open, src/commitments.rs:440-471): the quotient
// (P(x) - y_j0) / (x - j0) has values q_j = (y_j0 - y_j) / (j0 - j) at j != j0 and
// q_j0 = P'(j0) = (1 / w_j0) sum_{j != j0} w_j (y_j - y_j0) / (j0 - j) (barycentric derivative).
void lagrange_node_quotient_dev(Ctx *c, const Fr *y, size_t N, size_t j0, Fr *q) {
  TNS_PROF(c, "open_scan", 32.0 * 6 * N);
  const Fr *w = bary_weights(c, N, 0, N);
  Fr v;
  TNS_HIP(hipMemcpyAsync(&v, y + j0, sizeof(Fr), hipMemcpyDeviceToHost, c->stream));
  TNS_HIP(hipStreamSynchronize(c->stream));
  const Fr xs = from_u64<FrCfg>((uint64_t)j0);
  NodeSweep s = node_sweep_begin(c, xs, N, q, j0);
  k_node_finish<false><<<grid_for(s.T, 256, 1u << 30), 256, 0, c->stream>>>(xs, N, s.T, s.Tm, j0, v, q, s.icp,
                                                                            s.inverted, w, y,
                                                                            nullptr, q, s.sp);
  TNS_LAUNCH_CHECK();
  k_sum_reduce<<<1, 1024, 0, c->stream>>>(s.sp, s.T, s.dev + 1);
  TNS_LAUNCH_CHECK();
  k_node_quotient<<<grid_for(N, 256), 256, 0, c->stream>>>(y, v, N, q);  // q_j0 = (v - y_j0) * 0 = 0 for now
  TNS_LAUNCH_CHECK();
  Fr h[2], wj;
  TNS_HIP(hipMemcpyAsync(h, s.dev, sizeof h, hipMemcpyDeviceToHost, c->stream));
  TNS_HIP(hipMemcpyAsync(&wj, w + j0, sizeof(Fr), hipMemcpyDeviceToHost, c->stream));
  TNS_HIP(hipStreamSynchronize(c->stream));
  const Fr qj0 = mul(h[1], inv(wj));
  TNS_HIP(hipMemcpyAsync(q + j0, &qj0, sizeof(Fr), hipMemcpyHostToDevice, c->stream));
  TNS_HIP(hipStreamSynchronize(c->stream));
}

// Two vectors on the same nodes, opened at the same z (Twist: addresses and values): one
// batch inversion serves both.  parts = {ell, sum0, sum1}; inv receives the shared inverses.
// canon_inv: the inverses are written canonical (every chain inverse scaled by R^-1, the raw 1;
// the products along the chain keep the factor), for lagrange_quotient_finish2_dev's CI form;
// the sums then carry it too and are scaled back by R (the raw R^2) after the readback.
void lagrange_open_partial2_dev(Ctx *c, const Fr *y0, const Fr *y1, size_t N, size_t first, size_t cnt, const Fr &z,
                                Fr *inv, Fr parts[3], bool canon_inv, const std::function<void()> &queued) {
  TNS_PROF(c, "open_scan", 32.0 * 5 * cnt);  // pre write/read, inv write, y0, y1, w
  const Fr *w = bary_weights(c, N, first, cnt);
  const Fr xs = fr_shift(z, first);
  Fr scale = Fr::one();
  if (canon_inv) {
    scale = Fr::zero();
    scale.v[0] = 1;
  }
  NodeSweep s = node_sweep_begin(c, xs, cnt, inv, SIZE_MAX, scale, queued);
  k_node_finish2<<<grid_for(s.T, 256, 1u << 30), 256, 0, c->stream>>>(xs, cnt, s.T, s.Tm, inv, s.icp, s.inverted, scale,
                                                                      w, y0, y1, inv, s.sp);
  TNS_LAUNCH_CHECK();
  k_sum_reduce<<<1, 1024, 0, c->stream>>>(s.sp, s.T, s.dev + 1);
  TNS_LAUNCH_CHECK();
  k_sum_reduce<<<1, 1024, 0, c->stream>>>(s.sp + s.T, s.T, s.dev + 2);
  TNS_LAUNCH_CHECK();
  TNS_HIP(hipMemcpyAsync(parts, s.dev, 3 * sizeof(Fr), hipMemcpyDeviceToHost, c->stream));
  TNS_HIP(hipStreamSynchronize(c->stream));
  if (canon_inv) {
    Fr r2;
    for (int i = 0; i < 8; i++) r2.v[i] = FrCfg::R2[i];
    parts[1] = mul(parts[1], r2);
    parts[2] = mul(parts[2], r2);
  }
}

void lagrange_quotient_finish2_dev(Ctx *c, const Fr *y0, const Fr *y1, size_t cnt, const Fr &v0, const Fr &v1,
                                   const Fr *inv, Fr *q0, Fr *q1, unsigned *bits, bool canon_inv) {
  TNS_PROF(c, "open_scan", 32.0 * 5 * cnt);
  if (canon_inv && !bits) throw Error(TNS_ERR_INVALID_PARAMETERS, "canonical inverses give canonical quotients only");
  if (bits) {
    TNS_HIP(hipMemsetAsync(bits, 0, 2 * sizeof(unsigned), c->stream));
    auto kern = canon_inv ? k_node_quotient2_canon<true> : k_node_quotient2_canon<false>;
    kern<<<grid_for(cnt, 256), 256, 0, c->stream>>>(y0, y1, v0, v1, cnt, inv, q0, q1, bits);
  } else {
    k_node_quotient2<<<grid_for(cnt, 256), 256, 0, c->stream>>>(y0, y1, v0, v1, cnt, inv, q0, q1);
  }
  TNS_LAUNCH_CHECK();
}

void lagrange_quotient_finish_dev(Ctx *c, const Fr *y, size_t cnt, const Fr &v, Fr *q) {
  TNS_PROF(c, "open_scan", 32.0 * 3 * cnt);
  k_node_quotient<<<grid_for(cnt, 256), 256, 0, c->stream>>>(y, v, cnt, q);
  TNS_LAUNCH_CHECK();
}

}  // namespace tns
