// corun.hip -- can a memory-bound kernel with few VGPRs run in the register space a
// VALU-bound kernel leaves free (3 waves/SIMD at ~150 VGPRs: 56 left per SIMD lane)?
// k_valu mimics k_accumulate's occupancy (VGPRs ~150, no LDS, grid >> resident slots);
// k_copy streams HBM with few VGPRs.  Times each alone and both on two streams.
//   hipcc -O3 --offload-arch=gfx950 -o tools/corun tools/corun.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define NS 72
__global__ void __launch_bounds__(256) k_valu(uint32_t *out, int iters) {
  uint32_t s[NS];
#pragma unroll
  for (int i = 0; i < NS; i++) s[i] = threadIdx.x * 2654435761u + i * 40503u + blockIdx.x;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < NS; i++) {
      uint64_t p = (uint64_t)s[i] * s[(i + 1) % NS] + s[(i + 7) % NS];
      s[i] = (uint32_t)p ^ (uint32_t)(p >> 32);
    }
  }
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < NS; i++) x ^= s[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__global__ void __launch_bounds__(256) k_copy(const uint4 *__restrict__ in, uint4 *__restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = in[i];
}

int main(int argc, char **argv) {
  const int vblocks = 256 * 3 * 8, iters = argc > 1 ? atoi(argv[1]) : 200;
  const size_t bytes = (size_t)1 << 31, n = bytes / 16;
  const int cgrid = argc > 2 ? atoi(argv[2]) : 256 * 4;
  uint32_t *vo;
  uint4 *a, *b;
  (void)hipMalloc(&vo, sizeof(uint32_t) * vblocks * 256);
  (void)hipMalloc(&a, bytes);
  (void)hipMalloc(&b, bytes);
  (void)hipMemset(a, 1, bytes);
  hipStream_t s1, s2;
  (void)hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  hipEvent_t e[8];
  for (auto &x : e) (void)hipEventCreate(&x);
  float tv, tc, tv2, tc2;
  for (int rep = 0; rep < 3; rep++) {
    (void)hipEventRecord(e[0], s1);
    k_valu<<<vblocks, 256, 0, s1>>>(vo, iters);
    (void)hipEventRecord(e[1], s1);
    (void)hipEventSynchronize(e[1]);
    (void)hipEventElapsedTime(&tv, e[0], e[1]);
    (void)hipEventRecord(e[2], s2);
    for (int k = 0; k < 4; k++) k_copy<<<cgrid, 256, 0, s2>>>(a, b, n);
    (void)hipEventRecord(e[3], s2);
    (void)hipEventSynchronize(e[3]);
    (void)hipEventElapsedTime(&tc, e[2], e[3]);
    // both: the VALU kernel first, the copies queued behind it on the other stream
    (void)hipEventRecord(e[4], s1);
    k_valu<<<vblocks, 256, 0, s1>>>(vo, iters);
    (void)hipEventRecord(e[5], s1);
    (void)hipEventRecord(e[6], s2);
    for (int k = 0; k < 4; k++) k_copy<<<cgrid, 256, 0, s2>>>(a, b, n);
    (void)hipEventRecord(e[7], s2);
    (void)hipDeviceSynchronize();
    (void)hipEventElapsedTime(&tv2, e[4], e[5]);
    (void)hipEventElapsedTime(&tc2, e[6], e[7]);
    float span;
    (void)hipEventElapsedTime(&span, e[4], e[7]);
    printf("valu alone %.3f ms | copy alone %.3f ms (%.0f GB/s) | together: valu %.3f ms, copy %.3f ms (%.0f GB/s), copy ends %.3f ms after valu start\n",
           tv, tc, 4.0 * 2 * bytes / tc / 1e6, tv2, tc2, 4.0 * 2 * bytes / tc2 / 1e6, span);
  }
  return 0;
}
