// mad29bench.hip -- XYZZ mixed addition in radix 2^29 (csrc/f29.hpp, R' = 2^261) against the
// library's radix-2^32 lazy madd (bn254.hpp): the same chains of additions (every other point
// negated, as signed digits do), compared as affine points, and the throughput of both.
//   hipcc -O3 --offload-arch=gfx950 -o tools/mad29bench tools/mad29bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "f29.hpp"
using namespace tns;

__global__ void k_to_rp(const G1Affine *in, G1Affine *out, int n) {  // R -> R' (times 2^5), canonical
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fq c = from_u64<FqCfg>(32);
  G1Affine p = in[i];
  if (!p.is_inf()) {
    p.x = mul(p.x, c);
    p.y = mul(p.y, c);
  }
  out[i] = p;
}

// mode 0: random chains; 1: entry 1 repeats entry 0 (q = sum: the doubling); 2: entry 1 is
// -(entry 0) (the sum cancels to the identity, then goes on)
__device__ __forceinline__ int pick(int i, int k, int npts, int mode) {
  if (mode == 6) return (i * 64 + k) & (npts - 1);  // consecutive points (CURVE: (j + 1) G ascending)
  return (int)(((unsigned)i * 2654435761u + (unsigned)(mode && k == 1 ? 0 : k) * 40503u * 131u) & (unsigned)(npts - 1));
}
__device__ __forceinline__ bool negk(int i, int k, int mode) {
  if (mode == 4) return true;   // every point negated (a negative digit shared by a whole run)
  if (mode == 5) return false;
  if (mode == 1 && k == 1) k = 0;
  if (mode == 2 && k == 1) return !(i & 1);
  return (i + k) & 1;
}

__global__ void __launch_bounds__(256) k_ref(G1Xyzz *out, const G1Affine *pts, int iters, int npts, int dup) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  G1Xyzz acc = G1Xyzz::inf();
  for (int k = 0; k < iters; k++) {
    G1Affine q = pts[pick(i, k, npts, dup)];
    if (negk(i, k, dup) && !q.y.is_zero()) q.y = const_minus_dev<FqCfg, false>(q.y);
    acc = xyzz_madd_lazy(acc, q);
  }
  out[i] = xyzz_canon(acc);
}

__global__ void __launch_bounds__(256) k_r29(G1Xyzz *out, const G1Affine *pts, int iters, int npts, int dup) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  G1Xyzz29 acc;
  bool empty = true;
  for (int k = 0; k < iters; k++) {
    const G1Affine q = pts[pick(i, k, npts, dup)];
    xyzz_madd29(acc, empty, f29_from32(q.x), f29_from32(q.y), negk(i, k, dup) && !q.y.is_zero());
  }
  G1Xyzz r = G1Xyzz::inf();
  if (!empty) {
    r.x = f29_out(acc.x);
    r.y = f29_out(acc.y);
    r.zz = f29_out(acc.zz);
    r.zzz = f29_out(acc.zzz);
  }
  out[i] = xyzz_canon(r);
}

int main() {
  const int blocks = 256 * 8 * 2, n = blocks * 256;
  const int npts = getenv("NPTS_LOG") ? 1 << atoi(getenv("NPTS_LOG")) : 1 << 20;  // gather footprint
  std::vector<G1Affine> h(npts);
  uint64_t s = 88172645463325252ULL;
  for (auto &e : h)
    for (Fq *f : {&e.x, &e.y})
      for (int k = 0; k < 8; k++) {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        f->v[k] = (uint32_t)s & (k == 7 ? 0x0fffffffu : 0xffffffffu);
      }
  if (getenv("CURVE")) {  // real curve points: (i + 1) G for the first 4096, repeated
    G1Affine g;
    g.x = from_u64<FqCfg>(1);
    g.y = from_u64<FqCfg>(2);
    G1Xyzz acc = xyzz_from_affine(g);
    std::vector<G1Affine> cp(4096);
    const uint64_t tau = 0x9e3779b97f4a7c15ull;  // TAU: SRS-like tau^i G instead of (i + 1) G
    for (int i = 0; i < 4096; i++) {
      cp[i] = xyzz_to_affine(acc);
      acc = getenv("TAU") ? xyzz_mul_small(acc, tau) : xyzz_add(acc, xyzz_from_affine(g));
    }
    for (int i = 0; i < npts; i++) h[i] = cp[getenv("ASC") ? i % 4096 : (i * 2654435761u) % 4096];
  }
  G1Affine *pts, *pts29;
  G1Xyzz *o1, *o2;
  (void)hipMalloc(&pts, sizeof(G1Affine) * npts);
  (void)hipMalloc(&pts29, sizeof(G1Affine) * npts);
  (void)hipMalloc(&o1, sizeof(G1Xyzz) * n);
  (void)hipMalloc(&o2, sizeof(G1Xyzz) * n);
  (void)hipMemcpy(pts, h.data(), sizeof(G1Affine) * npts, hipMemcpyHostToDevice);
  k_to_rp<<<npts / 256, 256>>>(pts, pts29, npts);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int dup = 0; dup < 7; dup++) {
    const int it = dup >= 3 ? 400 : 40;  // modes 3-5: long chains (4: all negated, 5: none)
    const int nc = 4096;  // lanes compared
    std::vector<G1Xyzz> a(nc), b(nc);
    k_ref<<<blocks, 256>>>(o1, pts, it, npts, dup);
    k_r29<<<blocks, 256>>>(o2, pts29, it, npts, dup);
    (void)hipMemcpy(a.data(), o1, sizeof(G1Xyzz) * nc, hipMemcpyDeviceToHost);
    (void)hipMemcpy(b.data(), o2, sizeof(G1Xyzz) * nc, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int j = 0; j < nc; j++) {
      const G1Affine x = xyzz_to_affine(a[j]), y = xyzz_to_affine(b[j]);
      bad += !(x.x == y.x && x.y == y.y);
    }
    float t1, t2;
    (void)hipEventRecord(e0);
    k_ref<<<blocks, 256>>>(o1, pts, it, npts, dup);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&t1, e0, e1);
    (void)hipEventRecord(e0);
    k_r29<<<blocks, 256>>>(o2, pts29, it, npts, dup);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&t2, e0, e1);
    printf("mode %d: radix 2^32 lazy madd %6.2f G/s   radix 2^29 madd %6.2f G/s   mismatches %d/%d\n", dup,
           (double)n * it / t1 / 1e6, (double)n * it / t2 / 1e6, bad, nc);
  }
  return 0;
}
