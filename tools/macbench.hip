// macbench.hip -- issue cost and latency of the MSM's multiply-accumulate pattern on gfx950:
// v_mad_u64_u32 (+ v_addc_co_u32 carry) in independent streams vs dependent chains, at 1..8
// waves per SIMD.  Prints G instructions/s per kind; with the clock from a full-rate add
// stream this gives cycles per wave-instruction (issue cost) and the dependent latency.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/macbench.hip -o tools/macbench
#include <hip/hip_runtime.h>

#include <cstdio>

typedef unsigned long long ull;
typedef unsigned u32;

#define MAD(s) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(s) : "v"(a), "v"(b) : "vcc")
#define MADC(s, c) \
  asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc" : "+v"(s), "+v"(c) : "v"(a), "v"(b) : "vcc")
#define ADD(x) asm volatile("v_add_u32_e32 %0, %1, %0" : "+v"(x) : "v"(a))
#define MULLO(x) asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(x) : "v"(a))
#define MOV2(x, y) asm volatile("v_mov_b32_e32 %0, %1" : "=v"(x) : "v"(y))

// kind 0: 8 independent mads; 1: 8 independent mad+addc; 2: one dependent mad chain (8 per iter);
// 3: one dependent mad+addc chain; 4: 8 independent full-rate adds; 5: 2 chains of mad+addc;
// 6: 8 independent v_mul_lo_u32 (the Montgomery quotient digit m = t * INV)
template <int KIND>
__global__ void __launch_bounds__(64) k_bench(u32 *x, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const u32 a = x[i] | 1, b = x[i + 1] | 3;
  ull s0 = a, s1 = b, s2 = a ^ 1, s3 = b ^ 3, s4 = a + 5, s5 = b + 7, s6 = a * 3, s7 = b * 5;
  u32 c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0, c5 = 0, c6 = 0, c7 = 0;
  u32 y0 = a, y1 = b, y2 = a ^ 9, y3 = b ^ 7, y4 = a + 1, y5 = b + 2, y6 = a + 3, y7 = b + 4;
  for (int k = 0; k < iters; k++) {
    if (KIND == 0) { MAD(s0); MAD(s1); MAD(s2); MAD(s3); MAD(s4); MAD(s5); MAD(s6); MAD(s7); }
    if (KIND == 1) { MADC(s0, c0); MADC(s1, c1); MADC(s2, c2); MADC(s3, c3); MADC(s4, c4); MADC(s5, c5); MADC(s6, c6); MADC(s7, c7); }
    if (KIND == 2) { MAD(s0); MAD(s0); MAD(s0); MAD(s0); MAD(s0); MAD(s0); MAD(s0); MAD(s0); }
    if (KIND == 3) { MADC(s0, c0); MADC(s0, c0); MADC(s0, c0); MADC(s0, c0); MADC(s0, c0); MADC(s0, c0); MADC(s0, c0); MADC(s0, c0); }
    if (KIND == 4) { ADD(y0); ADD(y1); ADD(y2); ADD(y3); ADD(y4); ADD(y5); ADD(y6); ADD(y7); }
    if (KIND == 5) { MADC(s0, c0); MADC(s1, c1); MADC(s0, c0); MADC(s1, c1); MADC(s0, c0); MADC(s1, c1); MADC(s0, c0); MADC(s1, c1); }
    if (KIND == 6) { MULLO(y0); MULLO(y1); MULLO(y2); MULLO(y3); MULLO(y4); MULLO(y5); MULLO(y6); MULLO(y7); }
  }
  x[i] = (u32)(s0 ^ s1 ^ s2 ^ s3 ^ s4 ^ s5 ^ s6 ^ s7) + c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7 +
         (y0 ^ y1 ^ y2 ^ y3 ^ y4 ^ y5 ^ y6 ^ y7);
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
  return (double)blocks * 64 * iters * 8 / (ms * 1e6);  // G lane-instructions/s (mad+addc = 1)
}

int main() {
  u32 *d;
  hipMalloc(&d, sizeof(u32) * (256 * 4 * 8 * 64 + 64));
  hipMemset(d, 0x5a, sizeof(u32) * (256 * 4 * 8 * 64 + 64));
  const int it = 4000;
  printf("waves/SIMD | add x8 | mad x8 | mad+addc x8 | mad chain | mad+addc chain | 2 mad+addc chains | mul_lo x8  (G lane-ops/s)\n");
  for (int w : {1, 2, 3, 4, 6, 8}) {
    printf("%d | %.0f | %.0f | %.0f | %.0f | %.0f | %.0f | %.0f\n", w, run<4>(d, w, it), run<0>(d, w, it), run<1>(d, w, it),
           run<2>(d, w, it), run<3>(d, w, it), run<5>(d, w, it), run<6>(d, w, it));
  }
  return 0;
}
