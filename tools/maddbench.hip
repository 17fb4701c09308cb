// maddbench.hip -- library Fq product and XYZZ mixed addition (the MSM accumulation step)
// throughput on gfx950 for one build variant of the device arithmetic:
//   -DTNS_MONT_MUL_INC='"<file>"'  product variant (default: csrc/mont_mul.inc)
//   -DTNS_NO_FIELD_ASM             C add/sub/conditional subtraction instead of field_asm.inc
// Built here and run on the GPU box by tools/maddbench.sh; prints one line.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../multilinear-map-cryptography_amd/csrc/bn254.hpp"
using namespace tns;

__global__ void __launch_bounds__(256) k_mul(Fq *x, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  Fq a = x[2 * i], b = x[2 * i + 1];
  for (int k = 0; k < iters; k++) a = mul(a, b);
  x[2 * i] = a;
}

__global__ void __launch_bounds__(256) k_madd(G1Xyzz *acc_io, const G1Affine *pts, int iters, int npts) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  G1Xyzz acc = acc_io[i];
  for (int k = 0; k < iters; k++) acc = xyzz_madd(acc, pts[(i * 7 + k * 131) & (npts - 1)]);
  acc_io[i] = acc;
}

__global__ void __launch_bounds__(256) k_madd_lazy(G1Xyzz *acc_io, const G1Affine *pts, int iters, int npts) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  G1Xyzz acc = acc_io[i];
  for (int k = 0; k < iters; k++) acc = xyzz_madd_lazy(acc, pts[(i * 7 + k * 131) & (npts - 1)]);
  acc_io[i] = xyzz_canon(acc);
}

int main(int argc, char **argv) {
  const char *tag = argc > 1 ? argv[1] : "?";
  const int blocks = 256 * 8 * 2;
  const size_t n = (size_t)blocks * 256;
  std::vector<Fq> h(2 * n);
  uint64_t s = 88172645463325252ULL;
  for (auto &e : h) {
    for (int k = 0; k < 8; k++) {
      s ^= s << 13;
      s ^= s >> 7;
      s ^= s << 17;
      e.v[k] = (uint32_t)s;
    }
    e.v[7] &= 0x0fffffff;
  }
  Fq *d;
  (void)hipMalloc(&d, sizeof(Fq) * 2 * n);
  (void)hipMemcpy(d, h.data(), sizeof(Fq) * 2 * n, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int mit = 200;
  k_mul<<<blocks, 256>>>(d, 10);
  (void)hipEventRecord(e0);
  k_mul<<<blocks, 256>>>(d, mit);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float tm;
  (void)hipEventElapsedTime(&tm, e0, e1);
  std::vector<Fq> chk(4);
  (void)hipMemcpy(chk.data(), d, sizeof(Fq) * 4, hipMemcpyDeviceToHost);

  const int npts = 1 << 20;
  G1Affine *pts;
  G1Xyzz *accs;
  (void)hipMalloc(&pts, sizeof(G1Affine) * npts);
  (void)hipMemcpy(pts, h.data(), sizeof(G1Affine) * npts, hipMemcpyHostToDevice);
  (void)hipMalloc(&accs, sizeof(G1Xyzz) * n);
  (void)hipMemcpy(accs, h.data(), sizeof(G1Xyzz) * n / 2, hipMemcpyHostToDevice);
  const int ait = 40;
  k_madd<<<blocks, 256>>>(accs, pts, 2, npts);
  (void)hipEventRecord(e0);
  k_madd<<<blocks, 256>>>(accs, pts, ait, npts);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ta;
  (void)hipEventElapsedTime(&ta, e0, e1);
  // same start, lazy madd: the XYZZ representatives differ, the affine points must not
  std::vector<G1Xyzz> ref(256), lz(256);
  (void)hipMemcpy(accs, h.data(), sizeof(G1Xyzz) * n / 2, hipMemcpyHostToDevice);
  k_madd<<<blocks, 256>>>(accs, pts, ait, npts);
  (void)hipMemcpy(ref.data(), accs, sizeof(G1Xyzz) * 256, hipMemcpyDeviceToHost);
  (void)hipMemcpy(accs, h.data(), sizeof(G1Xyzz) * n / 2, hipMemcpyHostToDevice);
  (void)hipEventRecord(e0);
  k_madd_lazy<<<blocks, 256>>>(accs, pts, ait, npts);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float tl;
  (void)hipEventElapsedTime(&tl, e0, e1);
  (void)hipMemcpy(lz.data(), accs, sizeof(G1Xyzz) * 256, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int j = 0; j < 256; j++) {
    const G1Affine x = xyzz_to_affine(ref[j]), y = xyzz_to_affine(lz[j]);
    bad += !(x.x == y.x && x.y == y.y);
  }
  printf("%-14s mul %6.1f G/s   madd %6.2f G/s   lazy madd %6.2f G/s   lazy mismatches %d/256   check %08x\n", tag,
         (double)n * mit / tm / 1e6, (double)n * ait / ta / 1e6, (double)n * ait / tl / 1e6, bad,
         chk[0].v[0] ^ chk[1].v[3]);
  return 0;
}
