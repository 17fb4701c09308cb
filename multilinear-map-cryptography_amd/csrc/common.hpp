// common.hpp -- shared host-side plumbing for libtns: status codes, HIP error
// checks, grow-only device buffers, and the per-device context.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <cstdio>
#include <functional>
#include <map>
#include <condition_variable>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "../../include/tns.h"
#include "bn254.hpp"

namespace tns {

// A thrown tns::Error carries one of the TNS_* status codes of include/tns.h
// (mirroring TwistAndShoutError, src/lib.rs:59-78) across the C++ layer; the
// C-ABI entry points catch it and store the message for tns_last_error().
struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

void set_last_error(const std::string &msg);

#define TNS_HIP(call)                                                                  \
  do {                                                                                 \
    hipError_t _e = (call);                                                            \
    if (_e != hipSuccess)                                                              \
      throw ::tns::Error(TNS_ERR_DEVICE, std::string("HIP error ") + hipGetErrorString(_e) + \
                                             " at " __FILE__ ":" + std::to_string(__LINE__)); \
  } while (0)

#define TNS_LAUNCH_CHECK() TNS_HIP(hipGetLastError())

// Grow-only device allocation (never shrinks; freed with the context).
struct DevBuf {
  void *p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf &) = delete;
  DevBuf &operator=(const DevBuf &) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  void *ensure(size_t n) {
    if (n <= bytes && p) return p;
    release();
    size_t want = n ? n : 16;
    hipError_t e = hipMalloc(&p, want);
    if (e != hipSuccess) {
      p = nullptr;
      throw Error(TNS_ERR_OOM, "hipMalloc of " + std::to_string(want) + " bytes failed: " +
                                   hipGetErrorString(e));
    }
    bytes = want;
    return p;
  }
  template <class T>
  T *as() const {
    return reinterpret_cast<T *>(p);
  }
};

// Grow-only pinned host buffer (async device-to-host readbacks).
struct PinnedBuf {
  void *p = nullptr;
  size_t bytes = 0;
  PinnedBuf() = default;
  PinnedBuf(const PinnedBuf &) = delete;
  PinnedBuf &operator=(const PinnedBuf &) = delete;
  ~PinnedBuf() {
    if (p) (void)hipHostFree(p);
  }
  void *ensure(size_t n) {
    if (n <= bytes && p) return p;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    bytes = 0;
    hipError_t e = hipHostMalloc(&p, n ? n : 16, hipHostMallocDefault);
    if (e != hipSuccess) throw Error(TNS_ERR_OOM, std::string("hipHostMalloc failed: ") + hipGetErrorString(e));
    bytes = n ? n : 16;
    return p;
  }
};

// Grow-only fine-grained (coherent, device-mapped) host buffer: a kernel's last workgroup writes
// a small result and a flag here, and the host polls the flag instead of a stream synchronize.
struct MappedHostBuf {
  void *p = nullptr, *dev = nullptr;
  size_t bytes = 0;
  MappedHostBuf() = default;
  MappedHostBuf(const MappedHostBuf &) = delete;
  MappedHostBuf &operator=(const MappedHostBuf &) = delete;
  ~MappedHostBuf() {
    if (p) (void)hipHostFree(p);
  }
  void *ensure(size_t n) {
    if (n <= bytes && p) return p;
    if (p) (void)hipHostFree(p);
    p = dev = nullptr;
    bytes = 0;
    hipError_t e = hipHostMalloc(&p, n ? n : 64, hipHostMallocMapped | hipHostMallocCoherent);
    if (e != hipSuccess) throw Error(TNS_ERR_OOM, std::string("hipHostMalloc failed: ") + hipGetErrorString(e));
    e = hipHostGetDevicePointer(&dev, p, 0);
    if (e != hipSuccess) throw Error(TNS_ERR_DEVICE, std::string("hipHostGetDevicePointer: ") + hipGetErrorString(e));
    std::memset(p, 0, n ? n : 64);
    bytes = n ? n : 64;
    return p;
  }
};

// One stream's MSM workspaces (msm.hip): two lanes let two independent MSMs of a proof
// (the two commitments, the two opening quotients) overlap on the device.
struct MsmLane {
  hipStream_t stream = nullptr;
  DevBuf ws[19];
  DevBuf fix;       // heavy-bucket level sums
  // the lane's host readbacks without a stream synchronize: a one-block kernel copies the words
  // into this fine-grained host buffer and then sets the slot's flag, which the host polls
  // (lane_publish / lane_wait, msm.hip).  Slots: 0 scalar bit length, 1 the sort's last-pass
  // tile totals, 2 the MSM's per-set sums
  MappedHostBuf mapped;
  uint32_t pub_seq = 0;
  // the window plan this lane's last MSM of Montgomery scalars took (n, c, W, layout): the next
  // such MSM of n scalars counts pass 1 for it while it computes the scalars' bit length, and the
  // sort uses those counts when the bit length confirms the plan (bucket_sort_precount_bits)
  struct PlanHint {
    size_t n = 0;
    int c = 0, W = 0, bucket_bits = 0;
    bool shared = false;
  } hint;
  uint32_t slot_seq[3] = {0, 0, 0};
};
// (msm.hip) readbacks through MsmLane::mapped: parts (device pointer, bytes; bytes % 4 == 0) are
// copied back to back into the slot's data; lane_wait returns it once the flag shows the publish
constexpr int LANE_SLOT_BITS = 0, LANE_SLOT_SORT = 1, LANE_SLOT_SUMS = 2;
void lane_publish(MsmLane &ln, int slot, int n, const void *const *src, const size_t *bytes);
const void *lane_wait(MsmLane &ln, int slot);
// for kernels that publish themselves: the slot's data and flag (device views) and its new seq
void lane_publish_slot(MsmLane &ln, int slot, uint32_t **data, uint32_t **flag, uint32_t *seq);

// Per-level tables for exact interpolation on nodes {0..N-1} (interp.hip).
struct InterpPlan {
  unsigned log_n = 0;   // N = 2^log_n
  DevBuf fact, inv_fact;            // k!, 1/k!   (k < max(N, 2))
  DevBuf newton_kernel_hat;         // NTT_{2N}((-1)^t / t!), scaled by 1/(2N)
  DevBuf level_tables;              // per level: Vhat (2m) | Phat (2m)
  std::vector<size_t> level_off;    // element offset of level l (m = 2^l) in level_tables
};

// Window-shifted copies of a fixed point set for the shared-bucket MSM (msm.hip):
// table[j n + i] = 2^(c j) P_i, j < W.
struct FixedBase {
  DevBuf table;
  size_t n = 0;
  int c = 0, W = 0;
};

struct LagrangeBasis {
  DevBuf points;             // G1Affine[N]: G * L_j(tau)
  FixedBase *fb = nullptr;   // its window table (N >= 2^12)
  ~LagrangeBasis() { delete fb; }
};

struct Srs {
  DevBuf points;  // G1Affine[n]
  size_t n = 0;
  int device = 0;
  // setup_params keeps tau in CommitmentParams (src/utils.rs:94-100); with it the setup
  // also yields the Lagrange basis of the nodes {0..N-1}: G * L_j(tau) (lagrange.hip).
  bool has_tau = false;
  Fr tau;
  // (N, first node, node count) -> basis slice (cache)
  mutable std::map<std::tuple<size_t, size_t, size_t>, LagrangeBasis *> lagrange;
  size_t first = 0, held = 0;  // points[0..held) are g1_powers[first .. first + held) (sharded SRS)
  mutable FixedBase *fb = nullptr;                        // window table of `points` (lazy)
  Srs() = default;
  Srs(const Srs &) = delete;
  Srs &operator=(const Srs &) = delete;
  ~Srs() {
    for (auto &kv : lagrange) delete kv.second;
    delete fb;
  }
};

// Per-stage device time from HIP events recorded around the launches of one named stage
// (enabled by tns_profile_enable; used by bench.py for the roofline's live kernel duration).
// Besides the summed launch durations, each stage keeps the union of its launch intervals
// (stages of two MSM lanes overlap) and an optional operation count (MSM mixed additions).
struct KernelProfiler {
  bool enabled = false;
  hipEvent_t ref = nullptr;  // recorded at enable: common time origin of every stream
  struct Rec {
    std::string name;
    hipEvent_t a, b;
    double bytes;
  };
  struct Tot {
    double ms = 0, bytes = 0, ops = 0, busy_ms = 0;
    uint64_t launches = 0;
    std::vector<std::pair<double, double>> iv;
  };
  std::vector<Rec> pending;
  std::map<std::string, Tot> totals;
  std::string only;  // non-empty: time this stage alone
  void start(hipStream_t s) {
    reset();
    if (!ref) (void)hipEventCreate(&ref);
    (void)hipEventRecord(ref, s);
  }
  void reset() {
    collect();
    totals.clear();
  }
  void add_ops(const char *name, double ops) {
    if (enabled) totals[name].ops += ops;
  }
  void collect() {
    for (auto &r : pending) {
      float ms = 0.f, t0 = 0.f, t1 = 0.f;
      if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
        static const bool dbg = getenv("TNS_PROF_DEBUG") != nullptr;  // (diagnostics: read once)
        if (dbg) fprintf(stderr, "prof %s %.3f ms\n", r.name.c_str(), ms);
        auto &t = totals[r.name];
        t.ms += ms;
        t.launches += 1;
        t.bytes += r.bytes;
        if (ref && hipEventElapsedTime(&t0, ref, r.a) == hipSuccess && hipEventElapsedTime(&t1, ref, r.b) == hipSuccess)
          t.iv.emplace_back(t0, t1);
      }
      (void)hipEventDestroy(r.a);
      (void)hipEventDestroy(r.b);
    }
    pending.clear();
    for (auto &kv : totals) {  // union of the launch intervals
      auto &iv = kv.second.iv;
      std::sort(iv.begin(), iv.end());
      double busy = 0, lo = -1, hi = -1;
      for (auto &x : iv) {
        if (x.first > hi) {
          busy += hi - lo;
          lo = x.first;
          hi = x.second;
        } else if (x.second > hi) {
          hi = x.second;
        }
      }
      busy += hi - lo;
      kv.second.busy_ms = busy;
    }
  }
};

struct ProfScope {
  KernelProfiler *p = nullptr;
  hipStream_t s;
  KernelProfiler::Rec r;
  ProfScope(KernelProfiler &prof, hipStream_t st, const char *name, double alg_bytes) : s(st) {
    if (!prof.enabled || (!prof.only.empty() && prof.only != name)) return;
    p = &prof;
    r.name = name;
    r.bytes = alg_bytes;
    (void)hipEventCreate(&r.a);
    (void)hipEventCreate(&r.b);
    (void)hipEventRecord(r.a, s);
  }
  ~ProfScope() {
    if (!p) return;
    (void)hipEventRecord(r.b, s);
    p->pending.push_back(r);
  }
};

struct Ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;
  // workspaces
  DevBuf scratch[8];
  DevBuf sc_pong[4];    // sum-check: second fold buffer per table (the input tables stay intact)
  DevBuf sc_half[4], sc_chal, sc_out;  // the zero-closure fold chain on the side stream
  DevBuf sc_counter;                    // sum-check round kernel: last-workgroup counter
  DevBuf sc_poly;                       // ... and its composition (ScPoly, mle.hip)
  PinnedBuf sc_poly_host;               // (its host staging copy)
  MappedHostBuf sc_mapped;              // sum-check round results + flag, polled by the host
  MappedHostBuf sc_htab;                // sum-check: the folded tables of the host's last rounds
  MappedHostBuf inv_mapped;             // the batch inversion's grand product + flag (lagrange.hip)
  uint32_t inv_seq = 0;
  uint32_t sc_seq = 0;                  // the flag value of the latest round launch
  MappedHostBuf sc_handoff;             // sum-check challenges for pre-queued round kernels (host writes)
  DevBuf sc_rdev;                       // ... each copied to device memory by the waiting kernel
  DevBuf sc_tail_sync;                  // ... and relayed between the blocks of the persistent tail
  uint32_t sc_chal_seq = 0;             // the flag value of the latest published challenge
  PinnedBuf sc_host;    // its challenges (in) and bound table values (out)
  hipStream_t side = nullptr;  // the zero-closure folds
  hipStream_t copy = nullptr;  // host-buffer uploads that overlap a proof's first MSM (HostUpload)
  hipStream_t acc = nullptr;   // an MSM pair's accumulations (msm_pair_dev)
  PinnedBuf stage;             // their pinned staging ring (upload.cpp, built on first use)
  hipEvent_t stage_ev[32] = {};  // upload.cpp's staging ring: one event per slot
  DevBuf qbits;        // opening quotients' bit lengths (lagrange_quotient_finish2_dev)
  MsmLane lanes[2];     // lanes[0].stream == stream; lanes[1] has its own stream
  DevBuf prove_ws[12];  // resident trace / evaluation / quotient vectors of Twist/Shout::prove
  DevBuf twiddles;  // omega_{2^k}^i, i < 2^(k-1), natural order, for the largest k seen
  unsigned twiddle_log = 0;
  std::vector<InterpPlan *> plans;  // indexed by log_n
  std::map<uint32_t, DevBuf *> pass_tw;  // four-step pass twiddles keyed by (lo << 8 | r)
  std::map<std::tuple<size_t, size_t, size_t>, DevBuf *> bary_w;  // (N, first, count) -> weights
  bool lagrange_commit = true;           // prove via the Lagrange-basis SRS when available
  bool msm_tables = true;                // shared-bucket MSM on fixed bases with window tables
  int num_cu = 256;
  int upload_chunks = 4;  // drop-in provers: value-upload node ranges, each committed as it lands (tns_ctx_set_upload_chunks)
  KernelProfiler prof;
  ~Ctx();
};
// upload.cpp: host-to-device copies of the drop-in provers' inputs, in add() order on the
// context's copy stream from a helper thread (pinned staging ring, worker threads); wait(i, s)
// makes stream s wait for item i.  The destructor joins the thread and drains the copy stream.
class HostUpload {
 public:
  explicit HostUpload(Ctx *c);
  ~HostUpload();
  HostUpload(const HostUpload &) = delete;
  HostUpload &operator=(const HostUpload &) = delete;
  int add(void *dst, const void *src, size_t bytes);
  // n u64 values (trace addresses, lookup indices) sent packed into `small` (4 n bytes) as 24-bit
  // values (3 bytes each, four to three words) when every value is below 2^24, else as u32 when
  // every value fits 32 bits, else as they are into dst64; narrow_width(item) says which (3, 4 or
  // 8 bytes a value) once wait(item) has returned -- widen_dev expands the first two
  int add_narrow(uint32_t *small, uint64_t *dst64, const uint64_t *src, size_t n);
  int narrow_width(int item);
  void start();
  void wait(int item, hipStream_t s);
  void wait_all(hipStream_t s);

 private:
  struct Item {
    void *dst = nullptr;
    const void *src = nullptr;
    size_t bytes = 0;
    hipEvent_t ev = nullptr;
    bool narrow = false, done = false;
    int width = 8;  // bytes a value crossed PCIe as (narrow items)
    void *dst_wide = nullptr;
  };
  struct Job {  // one chunk of one item (or a whole small item: direct)
    int item;
    size_t off, cnt;  // source units: bytes, or u64 values for a narrow item
    bool direct;
  };
  struct ItemState {  // worker-side progress of an item
    std::atomic<size_t> left{0};
    std::atomic<bool> fits24{true}, fits32{true};
  };
  void run();
  void run_jobs();
  void work(int w, char *ring, std::atomic<size_t> &next, std::atomic<bool> &stop);
  hipError_t do_job(const Job &j, char *ring, int w, int &use);
  hipError_t finish_item(int k, char *ring, int w, int &use);
  hipError_t stage(char *ring, int w, int &use, void *dst, const void *src, size_t bytes);
  hipError_t stage_u32(char *ring, int w, int &use, uint32_t *dst, const uint64_t *src, size_t n);
  void mark_first();
  std::chrono::steady_clock::time_point t_start_, t_first_;
  std::atomic<bool> first_marked_{false};
  Ctx *c_;
  std::vector<Item> items_;
  std::vector<Job> jobs_;
  std::unique_ptr<ItemState[]> state_;
  std::thread th_;
  std::mutex mu_;
  std::condition_variable cv_;
  int queued_ = 0;
  bool done_ = false;
  hipError_t err_ = hipSuccess;
};

#define TNS_CAT2(a, b) a##b
#define TNS_CAT(a, b) TNS_CAT2(a, b)
// TNS_PROF(ctx, "stage", algorithmic_bytes_of_this_launch)
#define TNS_PROF(ctx, name, bytes) \
  ::tns::ProfScope TNS_CAT(_tns_prof_, __LINE__)((ctx)->prof, (ctx)->stream, name, (double)(bytes))
#define TNS_PROF_ON(ctx, stream, name, bytes) \
  ::tns::ProfScope TNS_CAT(_tns_prof_, __LINE__)((ctx)->prof, stream, name, (double)(bytes))

// RAII device guard + lock
struct CtxScope {
  Ctx *c;
  std::lock_guard<std::mutex> lk;
  explicit CtxScope(Ctx *ctx) : c(ctx), lk(ctx->mu) { TNS_HIP(hipSetDevice(ctx->device)); }
};

inline unsigned grid_for(size_t work, unsigned block, unsigned max_blocks = 4096) {
  size_t g = (work + block - 1) / block;
  if (g < 1) g = 1;
  if (g > max_blocks) g = max_blocks;
  return (unsigned)g;
}

inline unsigned ilog2_exact(size_t n) {
  unsigned l = 0;
  while (((size_t)1 << l) < n) l++;
  return l;
}

inline size_t next_pow2(size_t n) {  // Rust usize::next_power_of_two (0 -> 1)
  size_t p = 1;
  while (p < n) p <<= 1;
  return p;
}

// ---- module entry points (device-resident pointers; all on ctx->stream) ----
// mle.hip
void mle_fold_dev(Ctx *c, const Fr *in, Fr *out, size_t half, const Fr &r);
Fr mle_evaluate_dev(Ctx *c, const Fr *evals, unsigned nv, const Fr *point_host);
struct SumcheckTerm {
  Fr coeff;
  int tab[3];
};
// Runs every round of SumCheck::prove over k device tables of 2^nv entries
// (consumed: they are folded in place into workspace).  Transcript callback is
// host-side.  Returns status; fills rounds (nv x 4), challenges, final values.
struct HostTranscript;
// The zero-closure fold chain (mle.hip): binds the k tables at the challenges on stream st and
// writes their values to d_out.  flags (optional): the last table as 0/1 bytes (n_flags of
// them, zero beyond), tables[k - 1] unused -- only when sumcheck_folds_take_flag_bytes(nv).
bool sumcheck_folds_take_flag_bytes(unsigned nv);
void sumcheck_zero_folds_async(Ctx *c, hipStream_t st, Fr *const *tables, int k, unsigned nv, const Fr *chal_pinned,
                               Fr *d_out, const uint8_t *flags = nullptr, size_t n_flags = 0);
Fr composition_sum_dev(Ctx *c, Fr *const *tables, int k, unsigned nv, const SumcheckTerm *terms, int n_terms);
int sumcheck_prove_dev(Ctx *c, Fr *const *tables, int k, unsigned nv, const Fr &claimed,
                       const SumcheckTerm *terms, int n_terms, HostTranscript &tr, Fr *rounds,
                       Fr *challenges, Fr *final_table_values, Fr *final_eval);

// poly.hip
// q[i] = c[i+1] + z q[i+1] (synthetic division by x - z); returns P(z).  q may be null.
Fr synthetic_division_dev(Ctx *c, const Fr *coeffs, size_t n, const Fr &z, Fr *q);
// g1_powers[first .. first + n) = G * tau^i
void srs_generate_dev(Ctx *c, const Fr &tau, size_t first, size_t n, G1Affine *out);
void fr_fill_zero_dev(Ctx *c, Fr *p, size_t n);
// u64 entries [0, n_in) zero-padded to n: Montgomery form (mont), canonical form (canon,
// optional) and the largest bit length (*bits, zeroed here) in one pass on stream s
void u64_tables_dev(hipStream_t s, const uint64_t *in, size_t n_in, size_t n, Fr *mont, Fr *canon, unsigned *bits);
// out[i] = in[i] widened to u64 (addresses / indices that crossed PCIe as u32), on stream s
void widen_u32_dev(hipStream_t s, const uint32_t *in, size_t n, uint64_t *out);
// HostUpload narrow items: width 3 (packed 24-bit) or 4 (u32) -> u64 (width 8: nothing to do)
void widen_dev(hipStream_t s, const uint32_t *in, int width, size_t n, uint64_t *out);

// msm.hip (fb: optional window table of `points`, enabling the shared-bucket layout)
// fb_off: the points are entries [fb_off, fb_off + n) of the set fb was built for
G1Xyzz msm_dev(Ctx *c, const G1Affine *points, const Fr *scalars, size_t n, const FixedBase *fb = nullptr,
               size_t fb_off = 0);
// bit length of a canonical field element (0 for zero)
__device__ __forceinline__ unsigned fr_bit_length(const Fr &k) {
  unsigned b = 0;
#pragma unroll
  for (int l = 0; l < 8; l++)
    if (k.v[l]) b = 32 * l + 32 - __builtin_clz(k.v[l]);
  return b;
}
// max over the block of (b0, b1) -> one atomicMax per block and target (blockDim.x a multiple
// of 64, at most 1024; every thread of the block calls it).  A per-wave atomic on one address
// serialises in L2: 8 K of them were ~80 us of a 2^20-scalar bit-length pass.
__device__ __forceinline__ void block_atomic_max2(unsigned b0, unsigned b1, unsigned *dst0, unsigned *dst1) {
  __shared__ unsigned wmax[2][16];
  for (int o = 32; o > 0; o >>= 1) {
    b0 = max(b0, (unsigned)__shfl_xor(b0, o));
    b1 = max(b1, (unsigned)__shfl_xor(b1, o));
  }
  const int w = (int)(threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0) {
    wmax[0][w] = b0;
    wmax[1][w] = b1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < (int)(blockDim.x >> 6); i++) {
      b0 = max(b0, wmax[0][i]);
      b1 = max(b1, wmax[1][i]);
    }
    if (b0) atomicMax(dst0, b0);
    if (b1 && dst1) atomicMax(dst1, b1);
  }
}
struct MsmArgs {
  const G1Affine *points;
  const Fr *scalars;
  size_t n;
  const FixedBase *fb;
  // set: the scalars' largest bit length is at this device address and the sort reads
  // canonical scalars -- `canon` if set (then `scalars` stay Montgomery, for the tiny path),
  // else `scalars` themselves (n > 64 only: the tiny path reads Montgomery scalars)
  const unsigned *canon_bits = nullptr;
  const Fr *canon = nullptr;
  // set (with canon_bits, canonical scalars): pass 1's histograms are precounted (SortInput::precounted)
  const uint32_t *precounted = nullptr;
  int pre_c = 0, pre_W = 0;
  // > 0: plan the MSM for scalars of this bit length without reading canon_bits back (the opening
  // quotients: full width -- the table plan's extra windows of a narrower quotient carry no digits,
  // so the entries are the same); the sort can be queued right behind the kernel writing the scalars
  int plan_bits = 0;
  // set (with canon_bits): the sort reads these raw u64 values (entries [0, n_u64)) instead
  const uint64_t *u64 = nullptr;
  size_t n_u64 = 0;
  // enqueued on the lane's stream before anything else of this MSM: produces the scalars
  // (and canon / canon_bits) without holding up the other lane
  std::function<void(hipStream_t)> prep;
  // the scalars are still arriving (a host upload in flight; prep waits for it): msm_pair_dev
  // queues the other MSM whole before this one's prep
  bool late = false;
  // late and chunks > 1: the scalars arrive in `chunks` node ranges, chunk k = scalars
  // [chunk_off[k], chunk_off[k + 1]), ready once chunk_prep(k, stream) returns; msm_pair_dev sums
  // one MSM per chunk as each lands (table plans use the window table at the chunk's offset), so
  // only the last chunk's MSM follows the upload
  int chunks = 0;
  std::vector<size_t> chunk_off;  // chunks + 1 offsets, increasing, chunk_off[chunks] = n
  std::function<void(int, hipStream_t)> chunk_prep;
};
// how one vector of commit_evals_pair gets ready (the MsmArgs fields of the same names)
struct ScalarSource {
  std::function<void(hipStream_t)> prep;
  bool late = false;
  int chunks = 0;                                   // (MsmArgs::chunks, chunk_off, chunk_prep)
  std::vector<size_t> chunk_off;
  std::function<void(int, hipStream_t)> chunk_prep;
  const Fr *canon = nullptr;
  const unsigned *canon_bits = nullptr;
  const uint64_t *u64 = nullptr;
  size_t n_u64 = 0;
};
// two independent MSMs overlapped on the context's two lanes (inputs ready on c->stream)
void msm_pair_dev(Ctx *c, const MsmArgs &a, const MsmArgs &b, G1Xyzz out[2]);
// bucket_sort.hip: the MSM's digit entries grouped by bucket (bucket k = [bstart[k], bstart[k+1]))
struct BucketOrder {
  uint32_t *keys, *vals, *bstart;  // keys == nullptr: packed tail, the runs come from bstart alone
  int ks;          // bucket = key >> ks
  size_t entries;  // sorted entries (non-zero digits) when read back, else SIZE_MAX
};
// What the bucket sort's digit pass reads: canonical scalars, Montgomery scalars (converted in
// the pass: no canonical copy is written), or raw u64 values (trace addresses, lookup indices:
// 8 bytes a scalar instead of 32; entries [0, n_u64), zero above).
struct SortInput {
  const Fr *fr = nullptr;
  bool mont = false;
  const uint64_t *u64 = nullptr;
  size_t n_u64 = 0;
  // set: pass 1's tile histograms are already in the lane's count buffer (== precounted), computed
  // for the shared-table plan (pre_c, pre_W) over these n scalars (quotient2_count_dev: the opening
  // quotients' kernel counts their digits as it writes them); another plan recounts
  const uint32_t *precounted = nullptr;
  int pre_c = 0, pre_W = 0;
  bool pre_shared = true;
  // set (with precounted, Montgomery scalars): the count kernel also wrote each scalar's canonical
  // low 64 bits here; when the bit length shows the scalars fit 64 bits the sort reads these
  // (8 bytes a scalar, no Montgomery reduction) instead of the 32-byte scalars
  const uint64_t *low64 = nullptr;
};
// A sort in flight: bucket_sort_begin (pass 1), bucket_sort_passes (the passes up to the last
// pass's tile-total readback), bucket_sort_finish (waits for that readback, queues the rest);
// all but the wait are queued on the lane without blocking the host.
struct BucketSortJob {
  MsmLane *ln = nullptr;
  size_t E = 0, S = 0;
  int bucket_bits = 0, wb = 0, npass = 0, cur = 0, nb = 0, shift = 0, tile = 0, keybits = 0;
  int bits[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // key bits per pass
  bool last = false, pending = false;
  const void *readback = nullptr;  // the last pass's tile totals once read back (host memory)
  uint32_t *K[2] = {nullptr, nullptr}, *V[2] = {nullptr, nullptr}, *seg[2] = {nullptr, nullptr};
  uint32_t *counts = nullptr, *offs = nullptr, *tcount = nullptr, *tbase = nullptr, *desc = nullptr;
  uint32_t *mcount = nullptr, *mbase = nullptr;
  uint32_t *valid = nullptr;  // device: the entry count
  // packed tail (pk): the second-to-last pass writes one u32 per entry -- the last pass's key
  // bits, the sign and the point index i (ibits bits) -- and the last pass reads that word and
  // writes the accumulation's values only (no keys: runs come from the bucket starts)
  bool pk = false, vo = false, shared = false;  // vo: the last pass writes values only
  int ibits = 0, p = 0;
  uint32_t stride = 0;
  int kf[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // key format pass p writes (bucket_sort.hip KF_*)
};
void bucket_sort_begin(MsmLane &ln, const SortInput &in, size_t n, int c, int W, bool shared, uint32_t stride,
                       int bucket_bits, uint32_t *valid, BucketSortJob &J);
void bucket_sort_passes(BucketSortJob &J);
void bucket_sort_pass_rest(BucketSortJob &J, bool readback);
BucketOrder bucket_sort_finish(BucketSortJob &J);
// both phases at once (single MSMs)
// The two opening MSMs' scalars q_k,i = (v_k - y_k,i) inv_i (canonical: the inverses are) with their
// bit lengths, as lagrange_quotient_finish2_dev, AND pass 1's tile histograms of both sorts for the
// shared-table plan (c, W) straight into lanes[0] / lanes[1]'s count buffers: the sorts skip their
// count kernels (one read of both quotient vectors less).  false (nothing queued): no compile-time
// pass-1 plan for (c, W) -- the caller runs the plain quotient kernel.
bool quotient2_count_dev(Ctx *c, const Fr *y0, const Fr *y1, size_t n, const Fr &v0, const Fr &v1, const Fr *inv,
                         Fr *q0, Fr *q1, unsigned *bits, int cw, int W, const uint32_t *counts_out[2]);
// n Montgomery scalars' largest bit length (into *bits, zeroed by the caller) together with pass 1's
// histograms for the plan (c, W, shared, bucket_bits) in the lane's count buffer; `in` then carries
// them as precounted.  false (nothing queued): no compile-time pass-1 plan for it.
bool bucket_sort_precount_bits(MsmLane &ln, const Fr *scalars, size_t n, int c, int W, bool shared, int bucket_bits,
                               unsigned *bits, SortInput &in, bool want_low64);
BucketOrder bucket_sort_dev(MsmLane &ln, const SortInput &in, size_t n, int c, int W, bool shared, uint32_t stride,
                            int bucket_bits, uint32_t *valid);
FixedBase *fixed_base_build_dev(Ctx *c, const G1Affine *points, size_t n);
// the same, or nullptr when the table does not fit in device memory (TNS_ERR_OOM)
FixedBase *fixed_base_try_build(Ctx *c, const G1Affine *points, size_t n);
// the SRS's window table, built on first use by an MSM of >= 2^16 points (nullptr below)
const FixedBase *srs_fixed_base(Ctx *c, const Srs &srs, size_t n);

// interp.hip
void interpolate_consecutive_dev(Ctx *c, const Fr *y, size_t n, Fr *coeffs);
void factorial_tables_dev(Ctx *c, size_t nf, Fr *fact, Fr *ifact);

// poly.hip: out[i] = G * s_i (affine), scalars canonical
void fixed_base_mul_dev(Ctx *c, const Fr *scalars_canon, size_t n, G1Affine *out);
void xyzz_to_affine_batch_dev(Ctx *c, const G1Xyzz *in, size_t n, G1Affine *out, Fq *prefix_scratch);

// lagrange.hip: KZG on evaluations over the nodes {0..N-1}, for the node slice
// [first, first + cnt) a rank holds (first = 0, cnt = N unsharded).
// Basis slice G * L_j(tau) (cached in srs); nullptr when srs has no tau or tau is a node.
const LagrangeBasis *lagrange_basis_dev(Ctx *c, const Srs &srs, size_t N, size_t first, size_t cnt);
// inv[i] = 1 / (z - j) (j = first + i); ell_part = prod (z - j); sum_part = sum w_j y_j / (z - j)
// over the slice.  P(z) = (prod of all ell parts) * (sum of all sum parts).  z not a node.
void lagrange_open_partial_dev(Ctx *c, const Fr *y, size_t N, size_t first, size_t cnt, const Fr &z, Fr *inv,
                               Fr *ell_part, Fr *sum_part);
// q_i = (v - y_i) * inv_i in place: the quotient's values on the slice
void lagrange_quotient_finish_dev(Ctx *c, const Fr *y, size_t cnt, const Fr &v, Fr *q);
// canon_inv: inv receives the inverses in canonical form (for the CI quotient kernel)
// queued (optional): run on the host once the pass's first kernels are queued, before its first
// host wait (side-stream work that should not delay the pass)
void lagrange_open_partial2_dev(Ctx *c, const Fr *y0, const Fr *y1, size_t N, size_t first, size_t cnt, const Fr &z,
                                Fr *inv, Fr parts[3], bool canon_inv = false,
                                const std::function<void()> &queued = nullptr);
// bits != nullptr: q0 / q1 come out CANONICAL with their largest bit lengths in bits[0..1];
// canon_inv (requires bits): inv holds canonical inverses (lagrange_open_partial2_dev's canon_inv)
void lagrange_quotient_finish2_dev(Ctx *c, const Fr *y0, const Fr *y1, size_t cnt, const Fr &v0, const Fr &v1,
                                   const Fr *inv, Fr *q0, Fr *q1, unsigned *bits, bool canon_inv = false);
// quotient values for an opening AT the node j0 (value y_j0), unsharded
void lagrange_node_quotient_dev(Ctx *c, const Fr *y, size_t N, size_t j0, Fr *q);
bool fr_is_node(const Fr &x, size_t N);
// barycentric weights w_j = (-1)^(N-1-j) / (j! (N-1-j)!) of the nodes [first, first + cnt) (cached)
const Fr *bary_weights_dev(Ctx *c, size_t N, size_t first, size_t cnt);
// tfree.hip: the Lagrange basis [L_j(tau)]G, j < N, from g1_powers[0..N) alone (no tau); cached in
// srs.lagrange under (N, 0, N) like the tau-derived one
const LagrangeBasis *lagrange_basis_from_powers_dev(Ctx *c, const Srs &srs, size_t N);

// comm.cpp: the exchange steps of a sharded proof
struct Comm {
  int rank = 0, size = 1;
  // deadline of one exchange (RCCL: polled on the stream, then ncclCommAbort; a host callback
  // enforces its own and returns non-zero), exchange counter and latency statistics
  double timeout_s = 600.0;
  uint64_t seq = 0;
  double total_s = 0.0, max_s = 0.0;
  double bytes_total = 0.0, bytes_max = 0.0;  // this rank's bytes per exchange step
  virtual ~Comm() = default;
  // 0 = one rank (self), 1 = host callback, 2 = RCCL
  virtual int kind() const = 0;
  // the rank count the transport itself reports (ncclCommCount for RCCL)
  virtual int seen_size() const { return size; }
  // every rank's `bytes` from `send`, in rank order, into recv (size * bytes)
  virtual void allgather(Ctx *c, const void *send, size_t bytes, void *recv) = 0;
  // one numbered, timed exchange step; a failure names this rank, the step and `what`
  void exchange(Ctx *c, const void *send, size_t bytes, void *recv, const char *what);
};
Comm &comm_self();
Comm *comm_callback_new(int rank, int size, tns_allgather_fn fn, void *user);
Comm *comm_rccl_new(Ctx *c, int rank, int size, const uint8_t uid[128]);
void comm_unique_id(uint8_t out[128]);
G1Xyzz allgather_sum_g1(Ctx *c, Comm &m, const G1Xyzz &part, const char *what);
std::vector<Fr> allgather_fr(Ctx *c, Comm &m, const Fr *part, size_t k, const char *what);

// pairing.cpp: BN254 G2 (D-type twist, affine over Fq2 = Fq[u]/(u^2+1)) and the pairing
struct G2Affine {
  Fq x0, x1, y0, y1;  // x = x0 + x1 u, y = y0 + y1 u
  bool inf = false;
};
G2Affine g2_generator();
G2Affine g2_add(const G2Affine &a, const G2Affine &b);
G2Affine g2_neg(const G2Affine &a);
G2Affine g2_mul(const G2Affine &a, const uint64_t k_canonical[4]);
bool g2_on_curve(const G2Affine &a);
bool pairing_eq(const G1Affine &P1, const G2Affine &Q1, const G1Affine &P2, const G2Affine &Q2);
void pairing_value(const G1Affine &P, const G2Affine &Q, Fq out[12]);

// verify.cpp: the reference verifiers (host)
G1Xyzz g1_mul_host(const G1Affine &P, const Fr &k);
G1Affine g1_generator_host();
void verifier_key(const Fr &tau, G1Affine *g1, G2Affine *g2, G2Affine *g2_tau);
bool kzg_verify_host(const G1Affine &g1, const G2Affine &g2, const G2Affine &g2_tau, const G1Affine &C,
                     const Fr &z, const Fr &v, const G1Affine &pi);
bool kzg_batch_verify_host(const G1Affine &g1, const G2Affine &g2, const G2Affine &g2_tau, size_t n,
                           const G1Affine *C, const Fr *z, const Fr *v, const G1Affine *pi);
struct HostTranscript;
bool protocol_verify_host(const G1Affine &g1, const G2Affine &g2, const G2Affine &g2_tau, const char *label0,
                          const char *label1, const G1Affine C[2], const Fr *rounds, unsigned nv,
                          const Fr &final_eval, unsigned n_openings, const G1Affine pi[2], const Fr vals[2]);

// serialize.cpp: ark-serialize 0.4 canonical encodings (host)
void g1_serialize(const G1Affine &P, bool compressed, uint8_t *out);
G1Affine g1_deserialize(const uint8_t *in, bool compressed, bool validate);
void fr_serialize(const Fr &x, uint8_t out[32]);
Fr fr_deserialize(const uint8_t in[32]);

// host-side helpers (transcript.cpp)
struct HostTranscript {
  std::vector<uint8_t> state;
  void append_label(const char *s);
  void append_bytes(const uint8_t *p, size_t n);
  void append_fr(const Fr &x);
  Fr challenge(const char *label);
  Fr challenge_bytes(const uint8_t *label, size_t n);
  // The next challenge's hash, started early: DefaultHasher writes the state's length FIRST, so no
  // hash state carries over between challenges -- but once the length the state will have at the
  // next challenge is known (a sum-check round appends fixed-size data), the SipHash blocks of the
  // bytes already in the state can run while the device computes the round; challenge() then
  // hashes only the round's own ~170 bytes.  Same hash, same challenge.
  void prehash(size_t final_len);
  struct Pre {
    bool valid = false;
    size_t final_len = 0, done = 0;  // bytes of the state absorbed (a multiple of 8)
    uint64_t v[4];
  } pre;
};
Fr commitment_hash(const G1Affine &a);
Fr host_fr_rand_chacha(const uint8_t seed[32], uint8_t *fs_seed_out /* nullable: next 32 bytes */);
uint64_t siphash13_keys00(const uint8_t *msg, size_t n);
void host_fr_rand_stream(const uint8_t seed[32], size_t n, Fr *out);
void chacha20_block_host(const uint32_t key[8], uint64_t counter, uint32_t out[16]);
// Lagrange interpolation of 4 points (0..3) for sum-check round polys (host, exact).
void interpolate4_host(const Fr e[4], Fr out[4]);
Fr horner_host(const Fr *c, int n, const Fr &z);

}  // namespace tns
