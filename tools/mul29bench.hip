// mul29bench.hip -- Fq Montgomery product in radix 2^29 (9 limbs, R = 2^261) vs the library's
// radix-2^32 product-scanning product: every column sum of <= 18 products of 29/30-bit limbs
// fits a 64-bit register, so each MAC is one v_mad_u64_u32 with no carry instruction.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../multilinear-map-cryptography_amd/csrc/bn254.hpp"
using namespace tns;

struct F29 {
  u32 v[9];
};
__constant__ u32 P29c[9] = {0x187cfd47u, 0x010460b6u, 0x1c72a34fu, 0x02d522d0u, 0x1585d978u,
                            0x02db40c0u, 0x00a6e141u, 0x0e5c2634u, 0x0030644eu};
constexpr u32 P29[9] = {0x187cfd47u, 0x010460b6u, 0x1c72a34fu, 0x02d522d0u, 0x1585d978u,
                        0x02db40c0u, 0x00a6e141u, 0x0e5c2634u, 0x0030644eu};
constexpr u32 PINV29 = 0x04866389u, MASK29 = (1u << 29) - 1;

__device__ __forceinline__ F29 mul29(const F29 &a, const F29 &b) {
  u32 m[9];
  F29 r;
  unsigned long long acc = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
#pragma unroll
    for (int i = (k > 8 ? k - 8 : 0); i <= (k < 8 ? k : 8); i++) acc += (unsigned long long)a.v[i] * b.v[k - i];
    if (k < 9) {
#pragma unroll
      for (int i = 0; i < k; i++) acc += (unsigned long long)m[i] * P29[k - i];
      m[k] = ((u32)acc * PINV29) & MASK29;
      acc += (unsigned long long)m[k] * P29[0];
    } else {
#pragma unroll
      for (int i = k - 8; i < 9; i++) acc += (unsigned long long)m[i] * P29[k - i];
      r.v[k - 9] = (u32)acc & MASK29;
    }
    acc >>= 29;
  }
  r.v[8] = (u32)acc;
  return r;
}

__global__ void __launch_bounds__(256) k_mul29(F29 *x, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  F29 a = x[2 * i], b = x[2 * i + 1];
  for (int k = 0; k < iters; k++) a = mul29(a, b);
  x[2 * i] = a;
}
__global__ void __launch_bounds__(256) k_mul32(Fq *x, int iters) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  Fq a = x[2 * i], b = x[2 * i + 1];
  for (int k = 0; k < iters; k++) a = mul_lazy_dev(a, b);
  x[2 * i] = a;
}

int main() {
  const int blocks = 256 * 8 * 2;
  const size_t n = (size_t)blocks * 256;
  std::vector<F29> h(2 * n);
  uint64_t s = 88172645463325252ULL;
  for (auto &e : h)
    for (int k = 0; k < 9; k++) {
      s ^= s << 13;
      s ^= s >> 7;
      s ^= s << 17;
      e.v[k] = (u32)s & (k == 8 ? 0x1fffffu : MASK29);
    }
  F29 *d;
  (void)hipMalloc(&d, sizeof(F29) * 2 * n);
  (void)hipMemcpy(d, h.data(), sizeof(F29) * 2 * n, hipMemcpyHostToDevice);
  Fq *d32;
  (void)hipMalloc(&d32, sizeof(Fq) * 2 * n);
  (void)hipMemcpy(d32, h.data(), sizeof(Fq) * 2 * n, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int it = 200;
  float t29, t32;
  k_mul29<<<blocks, 256>>>(d, 5);
  (void)hipEventRecord(e0);
  k_mul29<<<blocks, 256>>>(d, it);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&t29, e0, e1);
  k_mul32<<<blocks, 256>>>(d32, 5);
  (void)hipEventRecord(e0);
  k_mul32<<<blocks, 256>>>(d32, it);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  (void)hipEventElapsedTime(&t32, e0, e1);
  printf("mul radix 2^29: %.1f G/s   radix 2^32 (lazy lib): %.1f G/s\n", (double)n * it / t29 / 1e6,
         (double)n * it / t32 / 1e6);
  return 0;
}
