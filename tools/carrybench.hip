// carrybench.hip -- does the carry register matter?  v_mad_u64_u32 + v_addc_co_u32 pairs with
// the carry in VCC (every pair serialised through one register) vs each pair's own SGPR pair,
// for independent streams and for the product-scanning column shape (one 64-bit accumulator
// chain + a carry word).  Prints G lane-pairs/s per kind at 1..8 waves per SIMD.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/carrybench.hip -o tools/carrybench
#include <hip/hip_runtime.h>

#include <cstdio>

typedef unsigned long long ull;
typedef unsigned u32;

#define MADC_VCC(s, c) \
  asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc" : "+v"(s), "+v"(c) : "v"(a), "v"(b) : "vcc")
#define MADC_S2(s, c, P, Q) \
  asm volatile("v_mad_u64_u32 %0, s[" #P ":" #Q "], %2, %3, %0\n\tv_addc_co_u32_e64 %1, s[" #P ":" #Q "], 0, %1, s[" #P ":" #Q "]" \
               : "+v"(s), "+v"(c) : "v"(a), "v"(b) : "s" #P, "s" #Q)
#define MADC_S(s, c, P) MADC_S_##P(s, c)
#define MADC_S_20(s, c) MADC_S2(s, c, 20, 21)
#define MADC_S_22(s, c) MADC_S2(s, c, 22, 23)
#define MADC_S_24(s, c) MADC_S2(s, c, 24, 25)
#define MADC_S_26(s, c) MADC_S2(s, c, 26, 27)
#define MADC_S_28(s, c) MADC_S2(s, c, 28, 29)
#define MADC_S_30(s, c) MADC_S2(s, c, 30, 31)
#define MADC_S_32(s, c) MADC_S2(s, c, 32, 33)
#define MADC_S_34(s, c) MADC_S2(s, c, 34, 35)

// kinds: 0 independent x8 via vcc; 1 independent x8, own SGPR pairs; 2 column chain (one acc) via vcc;
// 3 column chain, rotating 4 SGPR pairs; 4 two column chains interleaved via vcc; 5 two chains, own pairs
template <int KIND>
__global__ void __launch_bounds__(64) k_bench(u32 *x, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const u32 a = x[i] | 1, b = x[i + 1] | 3;
  ull s0 = a, s1 = b, s2 = a ^ 1, s3 = b ^ 3, s4 = a + 5, s5 = b + 7, s6 = a * 3, s7 = b * 5;
  u32 c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0, c5 = 0, c6 = 0, c7 = 0;
  for (int k = 0; k < iters; k++) {
    if (KIND == 0) { MADC_VCC(s0, c0); MADC_VCC(s1, c1); MADC_VCC(s2, c2); MADC_VCC(s3, c3); MADC_VCC(s4, c4); MADC_VCC(s5, c5); MADC_VCC(s6, c6); MADC_VCC(s7, c7); }
    if (KIND == 1) { MADC_S(s0, c0, 20); MADC_S(s1, c1, 22); MADC_S(s2, c2, 24); MADC_S(s3, c3, 26); MADC_S(s4, c4, 28); MADC_S(s5, c5, 30); MADC_S(s6, c6, 32); MADC_S(s7, c7, 34); }
    if (KIND == 2) { MADC_VCC(s0, c0); MADC_VCC(s0, c0); MADC_VCC(s0, c0); MADC_VCC(s0, c0); MADC_VCC(s0, c0); MADC_VCC(s0, c0); MADC_VCC(s0, c0); MADC_VCC(s0, c0); }
    if (KIND == 3) { MADC_S(s0, c0, 20); MADC_S(s0, c0, 22); MADC_S(s0, c0, 24); MADC_S(s0, c0, 26); MADC_S(s0, c0, 20); MADC_S(s0, c0, 22); MADC_S(s0, c0, 24); MADC_S(s0, c0, 26); }
    if (KIND == 4) { MADC_VCC(s0, c0); MADC_VCC(s1, c1); MADC_VCC(s0, c0); MADC_VCC(s1, c1); MADC_VCC(s0, c0); MADC_VCC(s1, c1); MADC_VCC(s0, c0); MADC_VCC(s1, c1); }
    if (KIND == 5) { MADC_S(s0, c0, 20); MADC_S(s1, c1, 22); MADC_S(s0, c0, 24); MADC_S(s1, c1, 26); MADC_S(s0, c0, 28); MADC_S(s1, c1, 30); MADC_S(s0, c0, 32); MADC_S(s1, c1, 34); }
  }
  x[i] = (u32)(s0 ^ s1 ^ s2 ^ s3 ^ s4 ^ s5 ^ s6 ^ s7) + c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
}

template <int KIND>
static double run(u32 *d, int waves_per_simd, int iters) {
  const int blocks = 256 * 4 * waves_per_simd;  // one 64-thread block = one wave
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k_bench<KIND><<<blocks, 64>>>(d, iters);
  hipEventRecord(e0);
  k_bench<KIND><<<blocks, 64>>>(d, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return (double)blocks * 64 * iters * 8 / (ms * 1e6);
}

int main() {
  u32 *d;
  hipMalloc(&d, sizeof(u32) * (256 * 4 * 8 * 64 + 64));
  hipMemset(d, 0x5a, sizeof(u32) * (256 * 4 * 8 * 64 + 64));
  const int it = 4000;
  printf("waves/SIMD | indep vcc | indep own-sgpr | chain vcc | chain 4 sgpr | 2 chains vcc | 2 chains own   (G lane-pairs/s)\n");
  for (int w : {1, 2, 3, 4, 6, 8}) {
    printf("%d | %.0f | %.0f | %.0f | %.0f | %.0f | %.0f\n", w, run<0>(d, w, it), run<1>(d, w, it), run<2>(d, w, it),
           run<3>(d, w, it), run<4>(d, w, it), run<5>(d, w, it));
  }
  return 0;
}
