// h2dbench.hip -- host-to-device upload options for the drop-in prove (host trace buffers):
// pageable hipMemcpy, two pageable copies from two threads at once, hipHostRegister of the
// caller's buffer (+ its cost) then DMA, a pinned staging buffer filled by T host threads.
// Sizes: the C4 trace's value vector (512 MiB) and address vector (128 MiB).  One line each.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const size_t V = (size_t)512 << 20, A = (size_t)128 << 20;
  std::vector<char> hv(V), ha(A);
  for (size_t i = 0; i < V; i += 4096) hv[i] = (char)i;
  for (size_t i = 0; i < A; i += 4096) ha[i] = (char)i;
  void *dv, *da;
  CK(hipMalloc(&dv, V));
  CK(hipMalloc(&da, A));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  CK(hipMemcpy(dv, hv.data(), V, hipMemcpyHostToDevice));  // warm
  for (int rep = 0; rep < 2; rep++) {
    double t0 = now_ms();
    CK(hipMemcpyAsync(dv, hv.data(), V, hipMemcpyHostToDevice, s1));
    CK(hipStreamSynchronize(s1));
    double t1 = now_ms();
    printf("pageable 512 MiB: %.2f ms = %.1f GB/s\n", t1 - t0, V / (t1 - t0) / 1e6);
    // two pageable copies from two threads (values + addresses)
    t0 = now_ms();
    std::thread th([&]() {
      (void)hipSetDevice(0);
      (void)hipMemcpyAsync(dv, hv.data(), V, hipMemcpyHostToDevice, s2);
      (void)hipStreamSynchronize(s2);
    });
    CK(hipMemcpyAsync(da, ha.data(), A, hipMemcpyHostToDevice, s1));
    CK(hipStreamSynchronize(s1));
    double ta = now_ms();
    th.join();
    t1 = now_ms();
    printf("two threads: 128 MiB done at %.2f ms, 512 MiB at %.2f ms (%.1f GB/s together)\n", ta - t0, t1 - t0,
           (V + A) / (t1 - t0) / 1e6);
    // register the caller's buffer in place, DMA, unregister
    t0 = now_ms();
    CK(hipHostRegister(hv.data(), V, hipHostRegisterDefault));
    double tr = now_ms();
    CK(hipMemcpyAsync(dv, hv.data(), V, hipMemcpyHostToDevice, s1));
    CK(hipStreamSynchronize(s1));
    double tc = now_ms();
    CK(hipHostUnregister(hv.data()));
    t1 = now_ms();
    printf("hipHostRegister %.2f ms + DMA %.2f ms (%.1f GB/s) + unregister %.2f ms\n", tr - t0, tc - tr,
           V / (tc - tr) / 1e6, t1 - tc);
  }
  // pinned staging filled by T threads, DMA'd in chunks as they fill
  char *pin;
  CK(hipHostMalloc((void **)&pin, V, hipHostMallocDefault));
  for (int T : {1, 4, 8, 16}) {
    const size_t chunk = (size_t)32 << 20, nch = V / chunk;
    double t0 = now_ms();
    std::vector<std::thread> ws;
    std::vector<hipEvent_t> ev(nch);
    for (auto &e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    // chunks in order: each chunk split over T threads, then its DMA queued
    for (size_t c = 0; c < nch; c++) {
      ws.clear();
      const size_t per = chunk / T;
      for (int t = 0; t < T; t++)
        ws.emplace_back([&, c, t]() { memcpy(pin + c * chunk + t * per, hv.data() + c * chunk + t * per, per); });
      for (auto &w : ws) w.join();
      CK(hipMemcpyAsync((char *)dv + c * chunk, pin + c * chunk, chunk, hipMemcpyHostToDevice, s1));
    }
    CK(hipStreamSynchronize(s1));
    double t1 = now_ms();
    printf("pinned staging, %2d memcpy threads, 32 MiB chunks: %.2f ms = %.1f GB/s\n", T, t1 - t0,
           V / (t1 - t0) / 1e6);
    for (auto &e : ev) (void)hipEventDestroy(e);
  }
  double t0 = now_ms();
  CK(hipMemcpyAsync(dv, pin, V, hipMemcpyHostToDevice, s1));
  CK(hipStreamSynchronize(s1));
  double t1 = now_ms();
  printf("pinned DMA alone: %.2f ms = %.1f GB/s\n", t1 - t0, V / (t1 - t0) / 1e6);
  (void)hipHostFree(pin);
  return 0;
}
