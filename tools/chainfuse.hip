// chainfuse.hip -- root-cause probe for the per-block chain inversion that was fused into
// k_node_chain in commit df7fe42 and withdrawn.  Runs, on the same x and
// node count n with T = 131072 chains:
//   A: the withdrawn fused kernel (chain products + block batch inversion in one kernel),
//   B: today's k_node_chain + k_chain_inv (lagrange.hip),
// and checks icp[t] * cp[t] == 1 for both, icp_A == icp_B, and the device inverse of every
// block total against the host inverse.  Built here (hipcc), run on the GPU box; one line per n.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <string>
#include <vector>

#include "../multilinear-map-cryptography_amd/csrc/bn254.hpp"
using namespace tns;

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

// A: df7fe42's k_node_chain, verbatim in its logic
__global__ void __launch_bounds__(256) k_chain_fused(Fr x, size_t n, size_t T, Fr Tm, Fr *__restrict__ pre,
                                                     Fr *__restrict__ cp, Fr *__restrict__ icp, Fr *__restrict__ tot) {
  __shared__ Fr sh[256];
  __shared__ Fr inv_total;
  const int tid = threadIdx.x;
  const size_t t = blockIdx.x * (size_t)blockDim.x + tid;
  Fr acc = Fr::one();
  if (t < T) {
    Fr d = sub(x, from_u64<FrCfg>((uint64_t)t));
    for (size_t i = t; i < n; i += T) {
      pre[i] = acc;
      acc = mul(acc, d);
      d = sub(d, Tm);
    }
    cp[t] = acc;
  }
  Fr lo = acc, hi = acc;
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
  if (tid == 0) {
    inv_total = inv(hi);
    tot[blockIdx.x] = hi;
  }
  sh[tid] = lo;
  __syncthreads();
  const Fr before = tid ? sh[tid - 1] : Fr::one();
  __syncthreads();
  sh[tid] = hi;
  __syncthreads();
  const Fr after = tid < 255 ? sh[tid + 1] : Fr::one();
  if (t < T) icp[t] = mul(mul(before, after), inv_total);
}

// B: today's split form (lagrange.hip k_node_chain + k_chain_inv)
__global__ void __launch_bounds__(256) k_chain(Fr x, size_t n, size_t T, Fr Tm, Fr *__restrict__ pre,
                                               Fr *__restrict__ cp) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (t >= T) return;
  Fr d = sub(x, from_u64<FrCfg>((uint64_t)t));
  Fr acc = Fr::one();
  for (size_t i = t; i < n; i += T) {
    pre[i] = acc;
    acc = mul(acc, d);
    d = sub(d, Tm);
  }
  cp[t] = acc;
}

__global__ void __launch_bounds__(256) k_inv_split(const Fr *__restrict__ cp, size_t T, Fr *__restrict__ icp) {
  __shared__ Fr sh[256];
  __shared__ Fr inv_total;
  const int tid = threadIdx.x;
  const size_t t = blockIdx.x * (size_t)blockDim.x + tid;
  Fr a = t < T ? cp[t] : Fr::one();
  Fr lo = a, hi = a;
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
  if (tid == 0) inv_total = inv(hi);
  sh[tid] = lo;
  __syncthreads();
  const Fr before = tid ? sh[tid - 1] : Fr::one();
  __syncthreads();
  sh[tid] = hi;
  __syncthreads();
  const Fr after = tid < 255 ? sh[tid + 1] : Fr::one();
  if (t < T) icp[t] = mul(mul(before, after), inv_total);
}

// df7fe42's k_node_finish2 (reads the chain inverse icp) and its parent's (inverts cp itself)
template <bool ICP>
__global__ void __launch_bounds__(256) k_finish2(Fr x, size_t n, size_t T, Fr Tm, const Fr *pre,
                                                 const Fr *__restrict__ c, const Fr *__restrict__ w,
                                                 const Fr *__restrict__ y0, const Fr *__restrict__ y1, Fr *invs,
                                                 Fr *__restrict__ sp) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (t >= T) return;
  if (t >= n) {
    sp[t] = sp[T + t] = Fr::zero();
    return;
  }
  const size_t cnt = (n - 1 - t) / T;
  size_t i = t + cnt * T;
  Fr d = sub(x, from_u64<FrCfg>((uint64_t)i));
  Fr iv = ICP ? c[t] : inv(c[t]);
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

__global__ void k_fill(Fr *a, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    Fr v;
    uint32_t h = seed ^ (uint32_t)i * 0x9e3779b9u;
    for (int k = 0; k < 8; k++) {
      h ^= h << 13;
      h ^= h >> 17;
      h ^= h << 5;
      v.v[k] = h;
    }
    v.v[7] &= 0x0fffffffu;
    a[i] = v;
  }
}

// k_finish2<true> with a record of the first two iterations of chain t == 0 (dbg[0..7]:
// iv0, pre_i, inv_i, d, iv1 for iteration 0; then pre_i, inv_i, d for iteration 1)
__global__ void __launch_bounds__(256) k_finish2_dbg(Fr x, size_t n, size_t T, Fr Tm, const Fr *pre,
                                                     const Fr *__restrict__ c, const Fr *__restrict__ w,
                                                     const Fr *__restrict__ y0, const Fr *__restrict__ y1, Fr *invs,
                                                     Fr *__restrict__ sp, Fr *__restrict__ dbg) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (t >= T) return;
  const size_t cnt = (n - 1 - t) / T;
  size_t i = t + cnt * T;
  Fr d = sub(x, from_u64<FrCfg>((uint64_t)i));
  Fr iv = c[t];
  Fr s0 = Fr::zero(), s1 = Fr::zero();
  int it = 0;
  if (t == 0) dbg[0] = iv;
  for (;;) {
    const Fr p = pre[i];
    const Fr inv_i = mul(iv, p);
    if (t == 0 && it < 2) {
      dbg[1 + 4 * it] = p;
      dbg[2 + 4 * it] = inv_i;
      dbg[3 + 4 * it] = d;
    }
    iv = mul(iv, d);
    if (t == 0 && it < 2) dbg[4 + 4 * it] = iv;
    it++;
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

static std::string hex(const Fr &v) {
  char b[80];
  for (int k = 0; k < 8; k++) sprintf(b + 8 * k, "%08x", v.v[7 - k]);
  return std::string(b);
}

int main() {
  const size_t T = 131072;
  Fr x;  // an arbitrary Montgomery-form element < r
  const uint32_t xv[8] = {0x9e3779b9u, 0x7f4a7c15u, 0x2545f491u, 0x4f6cdd1du,
                          0x12345678u, 0x0badf00du, 0x5eed1234u, 0x0123abcdu};
  for (int i = 0; i < 8; i++) x.v[i] = xv[i];
  const Fr Tm = from_u64<FrCfg>((uint64_t)T);
  for (size_t n : {(size_t)1 << 17, (size_t)1 << 18, (size_t)1 << 20, (size_t)1 << 24}) {
    const size_t Tn = n < T ? n : T, nb = (Tn + 255) / 256;
    Fr *pre, *cpA, *cpB, *icpA, *icpB, *tot;
    CK(hipMalloc(&pre, sizeof(Fr) * n));
    CK(hipMalloc(&cpA, sizeof(Fr) * Tn));
    CK(hipMalloc(&cpB, sizeof(Fr) * Tn));
    CK(hipMalloc(&icpA, sizeof(Fr) * Tn));
    CK(hipMalloc(&icpB, sizeof(Fr) * Tn));
    CK(hipMalloc(&tot, sizeof(Fr) * nb));
    k_chain_fused<<<nb, 256>>>(x, n, Tn, Tm, pre, cpA, icpA, tot);
    CK(hipGetLastError());
    k_chain<<<nb, 256>>>(x, n, Tn, Tm, pre, cpB);
    k_inv_split<<<nb, 256>>>(cpB, Tn, icpB);
    CK(hipDeviceSynchronize());
    std::vector<Fr> hA(Tn), hB(Tn), iA(Tn), iB(Tn), ht(nb);
    CK(hipMemcpy(hA.data(), cpA, sizeof(Fr) * Tn, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hB.data(), cpB, sizeof(Fr) * Tn, hipMemcpyDeviceToHost));
    CK(hipMemcpy(iA.data(), icpA, sizeof(Fr) * Tn, hipMemcpyDeviceToHost));
    CK(hipMemcpy(iB.data(), icpB, sizeof(Fr) * Tn, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ht.data(), tot, sizeof(Fr) * nb, hipMemcpyDeviceToHost));
    size_t cp_diff = 0, badA = 0, badB = 0, ab = 0, first_badA = SIZE_MAX;
    for (size_t t = 0; t < Tn; t++) {
      cp_diff += hA[t] != hB[t];
      if (mul(hA[t], iA[t]) != Fr::one()) {
        badA++;
        if (first_badA == SIZE_MAX) first_badA = t;
      }
      badB += mul(hB[t], iB[t]) != Fr::one();
      ab += iA[t] != iB[t];
    }
    {  // the consumer: df7's finish2 (icp) vs the parent's (inv(cp)) on the same pre / y / w
      Fr *w, *y0, *y1, *p1, *p2, *sp1, *sp2;
      CK(hipMalloc(&w, sizeof(Fr) * n));
      CK(hipMalloc(&y0, sizeof(Fr) * n));
      CK(hipMalloc(&y1, sizeof(Fr) * n));
      CK(hipMalloc(&p1, sizeof(Fr) * n));
      CK(hipMalloc(&p2, sizeof(Fr) * n));
      CK(hipMalloc(&sp1, sizeof(Fr) * 2 * Tn));
      CK(hipMalloc(&sp2, sizeof(Fr) * 2 * Tn));
      k_fill<<<1024, 256>>>(w, n, 1);
      k_fill<<<1024, 256>>>(y0, n, 2);
      k_fill<<<1024, 256>>>(y1, n, 3);
      k_chain_fused<<<nb, 256>>>(x, n, Tn, Tm, p1, cpA, icpA, tot);
      CK(hipMemcpy(p2, p1, sizeof(Fr) * n, hipMemcpyDeviceToDevice));
      k_finish2<true><<<nb, 256>>>(x, n, Tn, Tm, p1, icpA, w, y0, y1, p1, sp1);
      k_finish2<false><<<nb, 256>>>(x, n, Tn, Tm, p2, cpA, w, y0, y1, p2, sp2);
      CK(hipDeviceSynchronize());
      std::vector<Fr> a1(n), a2(n), s1(2 * Tn), s2(2 * Tn);
      CK(hipMemcpy(a1.data(), p1, sizeof(Fr) * n, hipMemcpyDeviceToHost));
      CK(hipMemcpy(a2.data(), p2, sizeof(Fr) * n, hipMemcpyDeviceToHost));
      CK(hipMemcpy(s1.data(), sp1, sizeof(Fr) * 2 * Tn, hipMemcpyDeviceToHost));
      CK(hipMemcpy(s2.data(), sp2, sizeof(Fr) * 2 * Tn, hipMemcpyDeviceToHost));
      size_t dinv = 0, dsp = 0, first = SIZE_MAX;
      for (size_t i = 0; i < n; i++)
        if (a1[i] != a2[i]) {
          dinv++;
          if (first == SIZE_MAX) first = i;
        }
      for (size_t i = 0; i < 2 * Tn; i++) dsp += s1[i] != s2[i];
      printf("  finish2(icp) vs finish2(inv cp): inverses differ %zu (first %zd), partial sums differ %zu\n", dinv,
             first == SIZE_MAX ? (ssize_t)-1 : (ssize_t)first, dsp);
      if (n == ((size_t)1 << 18)) {  // which variant is right: host 1 / (x - i) for chain t = 0 (i = 0, T)
        std::vector<Fr> pre(n), hc(Tn), hi(Tn);
        k_chain_fused<<<nb, 256>>>(x, n, Tn, Tm, p1, cpA, icpA, tot);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(pre.data(), p1, sizeof(Fr) * n, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hc.data(), cpA, sizeof(Fr) * Tn, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hi.data(), icpA, sizeof(Fr) * Tn, hipMemcpyDeviceToHost));
        for (size_t i : {(size_t)0, T}) {
          const Fr want = inv(sub(x, from_u64<FrCfg>((uint64_t)i)));
          printf("  i=%zu: icp-variant %s, inv-variant %s\n", i, a1[i] == want ? "right" : "WRONG",
                 a2[i] == want ? "right" : "WRONG");
        }
        {  // the failing kernel's intermediate values for chain 0 against the host
          Fr *dd, *p3, *sp3;
          CK(hipMalloc(&dd, sizeof(Fr) * 16));
          CK(hipMalloc(&p3, sizeof(Fr) * n));
          CK(hipMalloc(&sp3, sizeof(Fr) * 2 * Tn));
          CK(hipMemcpy(p3, p1, sizeof(Fr) * n, hipMemcpyDeviceToDevice));  // p1 holds pre again
          k_finish2_dbg<<<nb, 256>>>(x, n, Tn, Tm, p3, icpA, w, y0, y1, p3, sp3, dd);
          CK(hipDeviceSynchronize());
          Fr g[16];
          CK(hipMemcpy(g, dd, sizeof(Fr) * 9, hipMemcpyDeviceToHost));
          const Fr d0 = sub(x, from_u64<FrCfg>((uint64_t)T)), iv0 = hi[0];
          const Fr iv1 = mul(iv0, d0), d1 = add(d0, Tm);
          printf("  dbg it0: iv0 %d pre %d inv %d d %d iv1 %d | it1: pre %d inv %d d %d iv2 %d\n", g[0] == iv0,
                 g[1] == pre[T], g[2] == mul(iv0, pre[T]), g[3] == d0, g[4] == iv1, g[5] == pre[0],
                 g[6] == mul(iv1, pre[0]), g[7] == d1, g[8] == mul(iv1, d1));
          std::vector<Fr> a3(n);
          CK(hipMemcpy(a3.data(), p3, sizeof(Fr) * n, hipMemcpyDeviceToHost));
          size_t dd3 = 0;
          for (size_t i = 0; i < n; i++) dd3 += a3[i] != a2[i];
          printf("  dbg kernel inverses differing from the inv(cp) kernel: %zu\n", dd3);
          // the failing kernel's inverse of node 0 (second iteration of chain 0) against candidates
          const Fr bad = a1[0], good = a2[0], one = Fr::one();
          printf("  node0 bad  %s\n  node0 good %s\n", hex(bad).c_str(), hex(good).c_str());
          const Fr cands[] = {iv0, mul(iv0, d0), mul(iv0, d1), mul(iv1, d1), mul(iv1, pre[T]), mul(iv0, pre[T]),
                              mul(mul(iv1, d1), one), add(iv1, Tm), sub(iv1, Tm), mul(iv0, x), mul(iv1, x)};
          for (int k = 0; k < (int)(sizeof cands / sizeof cands[0]); k++)
            if (cands[k] == bad) printf("  node0 bad == candidate %d\n", k);
          int same = 0;
          for (int k = 0; k < 8; k++) same += bad.v[k] == good.v[k];
          printf("  node0 limbs equal to the right value: %d of 8\n", same);
          // and node T (first iteration) plus a few more chains
          size_t firsts_bad = 0, seconds_bad = 0;
          for (size_t t = 0; t < Tn; t++) {
            firsts_bad += a1[t + T] != a2[t + T];
            seconds_bad += a1[t] != a2[t];
          }
          printf("  chains with a wrong last node %zu, wrong first node %zu\n", firsts_bad, seconds_bad);
          (void)hipFree(dd);
          (void)hipFree(p3);
          (void)hipFree(sp3);
        }
        printf("  cp[0]   %s\n  icp[0]  %s\n  inv(cp) %s\n  pre[0] %s pre[T] %s\n", hex(hc[0]).c_str(),
               hex(hi[0]).c_str(), hex(inv(hc[0])).c_str(), hex(pre[0]).c_str(), hex(pre[T]).c_str());
      }
      for (Fr *q : {w, y0, y1, p1, p2, sp1, sp2}) (void)hipFree(q);
    }
    size_t tot_bad = 0;  // block totals: the host product of the block's chain products
    for (size_t b = 0; b < nb; b++) {
      Fr p = Fr::one();
      for (size_t t = b * 256; t < (b + 1) * 256 && t < Tn; t++) p = mul(p, hA[t]);
      tot_bad += p != ht[b];
    }
    printf("n=2^%d T=%zu: cp A!=B %zu | icp*cp!=1 fused %zu (first t %zd) split %zu | icp A!=B %zu | block totals wrong %zu\n",
           __builtin_ctzll(n), Tn, cp_diff, badA, first_badA == SIZE_MAX ? (ssize_t)-1 : (ssize_t)first_badA, badB,
           ab, tot_bad);
    (void)hipFree(pre);
    (void)hipFree(cpA);
    (void)hipFree(cpB);
    (void)hipFree(icpA);
    (void)hipFree(icpB);
    (void)hipFree(tot);
  }
  return 0;
}
