// sortbench.hip -- (bucket key, point) pair sorts of the MSM's size on MI355X:
// rocPRIM onesweep at several radix widths, for E = 12 * 2^24 entries and 21/22-bit keys.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/sortbench.hip -o tools/sortbench
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));     \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

__global__ void k_fill(uint32_t *k, uint32_t *v, size_t n, int bits) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t x = i * 0x9E3779B97F4A7C15ull + 12345;
    x ^= x >> 31;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 29;
    k[i] = (uint32_t)x & ((1u << bits) - 1);
    v[i] = (uint32_t)i;
  }
}

template <unsigned RB, unsigned BS, unsigned IPT>
using Cfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                       rocprim::radix_sort_onesweep_config<rocprim::kernel_config<BS, IPT>,
                                                                           rocprim::kernel_config<BS, IPT>, RB,
                                                                           rocprim::block_radix_rank_algorithm::match>>;

template <class C>
float run(const char *name, uint32_t *k, uint32_t *v, uint32_t *k2, uint32_t *v2, size_t n, int end_bit) {
  size_t tb = 0;
  CK(rocprim::radix_sort_pairs<C>(nullptr, tb, k, k2, v, v2, n, 0, end_bit));
  void *tmp;
  CK(hipMalloc(&tmp, tb));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e9;
  for (int it = 0; it < 4; it++) {
    CK(hipEventRecord(a));
    CK(rocprim::radix_sort_pairs<C>(tmp, tb, k, k2, v, v2, n, 0, end_bit));
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (it && ms < best) best = ms;
  }
  // check sortedness of a sample
  std::vector<uint32_t> h(1 << 20);
  CK(hipMemcpy(h.data(), k2 + n / 2, sizeof(uint32_t) * h.size(), hipMemcpyDeviceToHost));
  bool ok = true;
  for (size_t i = 1; i < h.size(); i++) ok &= h[i - 1] <= h[i];
  printf("%-28s end_bit %2d  %8.3f ms  %6.1f G pairs/s  %s\n", name, end_bit, best, n / best / 1e6,
         ok ? "sorted" : "NOT SORTED");
  CK(hipFree(tmp));
  return best;
}

int main() {
  const size_t n = (size_t)12 << 24;
  uint32_t *k, *v, *k2, *v2;
  CK(hipMalloc(&k, n * 4));
  CK(hipMalloc(&v, n * 4));
  CK(hipMalloc(&k2, n * 4));
  CK(hipMalloc(&v2, n * 4));
  for (int bits : {21, 22}) {
    k_fill<<<4096, 256>>>(k, v, n, bits);
    CK(hipDeviceSynchronize());
    run<rocprim::default_config>("default", k, v, k2, v2, n, bits);
    run<Cfg<8, 512, 12>>("onesweep rb8 512x12", k, v, k2, v2, n, bits);
    run<Cfg<7, 512, 12>>("onesweep rb7 512x12", k, v, k2, v2, n, bits);
    run<Cfg<11, 512, 12>>("onesweep rb11 512x12", k, v, k2, v2, n, bits);
    run<Cfg<11, 1024, 8>>("onesweep rb11 1024x8", k, v, k2, v2, n, bits);
  }
  return 0;
}
