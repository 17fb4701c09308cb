// upload.cpp -- host-to-device copies of the drop-in provers' inputs (tns_twist_prove /
// tns_shout_prove on the caller's pageable buffers), overlapped with the proof's first MSM.
//
// All queued items are cut into 16 MiB chunks up front and ONE pool of kWorkers threads takes the
// chunks in item order: a worker memcpys (or, for a narrowed item, converts u64 -> u32) its chunk
// into the next of its pinned ring slots (the context's staging buffer) and DMAs it on the
// context's copy stream as soon as it is full.  tools/h2dbench.hip on the MI355X box: pinned DMAs
// sustain 52-54 GB/s of the link's 57.5, where one pageable hipMemcpy of 512 MiB took 9.5-24 ms
// (22-56 GB/s, box- and run-dependent) and registering the caller's buffer in place
// (hipHostRegister) cost 23-26 ms before its DMA.  Round 3 sent the items one after the other
// (16 MiB chunks, the pool re-formed per item): the link idled while the next item's first chunks
// were staged -- 1.3 ms before the first DMA (a 32 MB address chunk converted by one thread) and
// ~1 ms between items (profiles/r04_dropin_timeline.txt).  The shared pool keeps the link busy
// across item boundaries.  The worker that queues an item's last chunk records the item's event
// on the copy stream; wait() makes a stream wait for it, blocking the calling thread only until
// the event is recorded (the copies are queued), not until the bytes land.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "common.hpp"

namespace tns {

namespace {
// bytes per DMA (one ring slot): 16 MiB.  4 MiB DMAs ran the link at 34 GB/s instead of 52 (the
// per-copy overhead); a narrowed item's chunks carry 8 MiB (2 M values converted by one thread:
// the first DMA starts ~0.6 ms in instead of ~1.3 ms with 4 M values)
constexpr size_t kChunk = (size_t)16 << 20, kNarrowPer = (size_t)2 << 20;
constexpr int kWorkers = 8, kPerWorker = 2, kSlots = kWorkers * kPerWorker;
constexpr size_t kDirect = (size_t)1 << 20;  // smaller items: one pageable hipMemcpyAsync
static_assert(kSlots <= (int)(sizeof(Ctx::stage_ev) / sizeof(hipEvent_t)), "one event per ring slot");
}  // namespace

HostUpload::HostUpload(Ctx *c) : c_(c) {}

HostUpload::~HostUpload() {
  if (th_.joinable()) th_.join();
  (void)hipStreamSynchronize(c_->copy);
  for (auto &it : items_)
    if (it.ev) (void)hipEventDestroy(it.ev);
}

int HostUpload::add(void *dst, const void *src, size_t bytes) {
  Item it;
  it.dst = dst;
  it.src = src;
  it.bytes = bytes;
  TNS_HIP(hipEventCreateWithFlags(&it.ev, hipEventDisableTiming));
  items_.push_back(it);
  return (int)items_.size() - 1;
}

int HostUpload::add_narrow(uint32_t *small, uint64_t *dst64, const uint64_t *src, size_t n) {
  const int id = add(small, src, 8 * n);
  items_[id].narrow = true;
  items_[id].dst_wide = dst64;
  return id;
}

int HostUpload::narrow_width(int item) {
  std::lock_guard<std::mutex> lk(mu_);
  return items_[item].width;
}

// the staging ring: kSlots chunks of pinned memory and one event per slot (its last DMA)
static char *stage_ring(Ctx *c) {
  if (!c->stage_ev[0])
    for (int s = 0; s < kSlots; s++) TNS_HIP(hipEventCreateWithFlags(&c->stage_ev[s], hipEventDisableTiming));
  return (char *)c->stage.ensure(kChunk * kSlots);
}

// TNS_UPLOAD_TRACE=1: the host-side span of an upload on stderr (start -> first DMA queued ->
// last item queued), for the drop-in timeline
void HostUpload::mark_first() {
  bool expect = false;
  if (first_marked_.compare_exchange_strong(expect, true)) t_first_ = std::chrono::steady_clock::now();
}

void HostUpload::run() {
  // runs on its own thread: nothing may escape it (std::terminate would take down a process that
  // has initialised the GPU); a failure is recorded in err_ and surfaces in wait() as a status
  try {
    run_jobs();
  } catch (const std::bad_alloc &) {
    std::lock_guard<std::mutex> lk(mu_);
    err_ = hipErrorOutOfMemory;
  } catch (...) {
    std::lock_guard<std::mutex> lk(mu_);
    if (err_ == hipSuccess) err_ = hipErrorUnknown;
  }
  {
    std::lock_guard<std::mutex> lk(mu_);
    done_ = true;
  }
  cv_.notify_all();
  static const bool trace = [] {
    const char *e = getenv("TNS_UPLOAD_TRACE");
    return e && e[0] == '1';
  }();
  if (trace) {
    using us = std::chrono::duration<double, std::micro>;
    const auto t_end = std::chrono::steady_clock::now();
    fprintf(stderr, "[upload] %zu items, %zu jobs: first DMA queued at %.0f us, all queued at %.0f us\n",
            items_.size(), jobs_.size(), first_marked_ ? us(t_first_ - t_start_).count() : -1.0,
            us(t_end - t_start_).count());
  }
}

// bytes through worker w's next ring slot: wait for the slot's previous DMA, copy, DMA, record
hipError_t HostUpload::stage(char *ring, int w, int &use, void *dst, const void *src, size_t bytes) {
  const int slot = w * kPerWorker + use;
  use = (use + 1) % kPerWorker;
  char *buf = ring + (size_t)slot * kChunk;
  hipError_t e = hipEventSynchronize(c_->stage_ev[slot]);
  if (e != hipSuccess) return e;
  std::memcpy(buf, src, bytes);
  mark_first();
  e = hipMemcpyAsync(dst, buf, bytes, hipMemcpyHostToDevice, c_->copy);
  if (e == hipSuccess) e = hipEventRecord(c_->stage_ev[slot], c_->copy);
  return e;
}

hipError_t HostUpload::do_job(const Job &j, char *ring, int w, int &use) {
  const Item &it = items_[j.item];
  if (j.direct) {
    if (!it.bytes) return hipSuccess;
    // (a small narrow item goes over as it is)
    return hipMemcpyAsync(it.narrow ? it.dst_wide : it.dst, it.src, it.bytes, hipMemcpyHostToDevice, c_->copy);
  }
  if (!it.narrow) return stage(ring, w, use, (char *)it.dst + j.off, (const char *)it.src + j.off, j.cnt);
  // narrow: u64 values -> 24-bit values packed four to three words in the slot (chunk offsets are
  // multiples of 4 values); a value past 24 (32) bits clears the item's fits24 (fits32) flag --
  // the bytes sent are then wrong, and finish_item sends the u32 (u64) array instead
  const int slot = w * kPerWorker + use;
  use = (use + 1) % kPerWorker;
  uint32_t *o = (uint32_t *)(ring + (size_t)slot * kChunk);
  hipError_t e = hipEventSynchronize(c_->stage_ev[slot]);
  if (e != hipSuccess) return e;
  const uint64_t *in = (const uint64_t *)it.src + j.off;
  uint64_t any = 0;
  const size_t q = j.cnt / 4;
  for (size_t g = 0; g < q; g++) {
    const uint64_t a = in[4 * g], b = in[4 * g + 1], c = in[4 * g + 2], d = in[4 * g + 3];
    any |= a | b | c | d;
    o[3 * g] = (uint32_t)(a & 0xffffff) | (uint32_t)(b << 24);
    o[3 * g + 1] = (uint32_t)((b >> 8) & 0xffff) | (uint32_t)(c << 16);
    o[3 * g + 2] = (uint32_t)((c >> 16) & 0xff) | (uint32_t)(d << 8);
  }
  if (j.cnt % 4) {  // the item's last values: a zero-padded group
    uint64_t v[4] = {0, 0, 0, 0};
    for (size_t i = 4 * q; i < j.cnt; i++) v[i - 4 * q] = in[i];
    any |= v[0] | v[1] | v[2] | v[3];
    o[3 * q] = (uint32_t)(v[0] & 0xffffff) | (uint32_t)(v[1] << 24);
    o[3 * q + 1] = (uint32_t)((v[1] >> 8) & 0xffff) | (uint32_t)(v[2] << 16);
    o[3 * q + 2] = (uint32_t)((v[2] >> 16) & 0xff) | (uint32_t)(v[3] << 8);
  }
  if (any >> 24) state_[j.item].fits24.store(false, std::memory_order_relaxed);
  if (any >> 32) state_[j.item].fits32.store(false, std::memory_order_relaxed);
  mark_first();
  const size_t words = 3 * ((j.cnt + 3) / 4);
  e = hipMemcpyAsync((uint32_t *)it.dst + 3 * (j.off / 4), o, 4 * words, hipMemcpyHostToDevice, c_->copy);
  if (e == hipSuccess) e = hipEventRecord(c_->stage_ev[slot], c_->copy);
  return e;
}

// n u64 values as u32 through worker w's next ring slot (a narrow item's 32-bit fallback)
hipError_t HostUpload::stage_u32(char *ring, int w, int &use, uint32_t *dst, const uint64_t *src, size_t n) {
  const int slot = w * kPerWorker + use;
  use = (use + 1) % kPerWorker;
  uint32_t *o = (uint32_t *)(ring + (size_t)slot * kChunk);
  hipError_t e = hipEventSynchronize(c_->stage_ev[slot]);
  if (e != hipSuccess) return e;
  for (size_t i = 0; i < n; i++) o[i] = (uint32_t)src[i];
  e = hipMemcpyAsync(dst, o, 4 * n, hipMemcpyHostToDevice, c_->copy);
  if (e == hipSuccess) e = hipEventRecord(c_->stage_ev[slot], c_->copy);
  return e;
}

// item k's chunks are all queued (this worker queued the last one): the u64 fallback of a narrow
// item that did not fit, then the item's event; items complete in order for wait()
hipError_t HostUpload::finish_item(int k, char *ring, int w, int &use) {
  Item &it = items_[k];
  hipError_t e = hipSuccess;
  const bool chunked = it.bytes >= kDirect;
  int width = 8;
  if (it.narrow && chunked) {
    width = state_[k].fits24.load() ? 3 : state_[k].fits32.load() ? 4 : 8;
    const size_t n = it.bytes / 8, per = kChunk / 4;
    const uint64_t *src = (const uint64_t *)it.src;
    if (width == 4)  // (rare: memories or tables past 2^24 entries)
      for (size_t off = 0; off < n && e == hipSuccess; off += per)
        e = stage_u32(ring, w, use, (uint32_t *)it.dst + off, src + off, std::min(per, n - off));
    if (width == 8)
      for (size_t off = 0; off < it.bytes && e == hipSuccess; off += kChunk)
        e = stage(ring, w, use, (char *)it.dst_wide + off, (const char *)it.src + off, std::min(kChunk, it.bytes - off));
  }
  if (e == hipSuccess) e = hipEventRecord(it.ev, c_->copy);
  {
    std::lock_guard<std::mutex> lk(mu_);
    it.width = width;
    it.done = true;
    while (queued_ < (int)items_.size() && items_[queued_].done) queued_++;
    if (e != hipSuccess && err_ == hipSuccess) err_ = e;
  }
  cv_.notify_all();
  return e;
}

void HostUpload::work(int w, char *ring, std::atomic<size_t> &next, std::atomic<bool> &stop) {
  hipError_t e = hipSetDevice(c_->device);
  int use = 0;
  try {  // (a worker thread: nothing may escape it)
    while (e == hipSuccess && !stop.load(std::memory_order_relaxed)) {
      const size_t j = next.fetch_add(1);
      if (j >= jobs_.size()) break;
      e = do_job(jobs_[j], ring, w, use);
      if (e == hipSuccess && state_[jobs_[j].item].left.fetch_sub(1, std::memory_order_acq_rel) == 1)
        e = finish_item(jobs_[j].item, ring, w, use);
    }
  } catch (...) {
    e = hipErrorUnknown;
  }
  if (e != hipSuccess) {
    stop.store(true);
    std::lock_guard<std::mutex> lk(mu_);
    if (err_ == hipSuccess) err_ = e;
  }
}

void HostUpload::run_jobs() {
  const int ni = (int)items_.size();
  state_.reset(new ItemState[ni]);
  bool staged = false;
  for (int k = 0; k < ni; k++) {
    const Item &it = items_[k];
    if (it.bytes < kDirect) {
      jobs_.push_back(Job{k, 0, it.bytes, true});
      state_[k].left = 1;
      continue;
    }
    staged = true;
    const size_t unit = it.narrow ? 8 : 1, per = it.narrow ? kNarrowPer : kChunk;  // source units per chunk
    const size_t total = it.bytes / unit;
    // the first item's first chunks ramp up (1/8, 1/4, 1/2 of a chunk): the link starts as soon as
    // a small piece is staged instead of after a whole chunk's copy or conversion
    size_t n = 0, step = k == 0 ? per / 8 : per;
    for (size_t off = 0; off < total; off += step, n++, step = std::min(per, 2 * step))
      jobs_.push_back(Job{k, off, std::min(step, total - off), false});
    state_[k].left = n;
  }
  char *ring = nullptr;
  if (staged) {
    try {
      ring = stage_ring(c_);
    } catch (const Error &) {
      std::lock_guard<std::mutex> lk(mu_);
      err_ = hipErrorOutOfMemory;
      return;
    }
  }
  std::atomic<size_t> next{0};
  std::atomic<bool> stop{false};
  std::vector<std::thread> ws;
  const int nw = (int)std::min<size_t>(kWorkers, jobs_.size());
  try {
    for (int w = 1; w < nw; w++) ws.emplace_back([&, w]() { work(w, ring, next, stop); });
  } catch (...) {  // workers that could not start: the others take their chunks (slots stay per worker)
  }
  work(0, ring, next, stop);
  for (auto &t : ws) t.join();
}

void HostUpload::start() {
  t_start_ = std::chrono::steady_clock::now();
  th_ = std::thread([this]() { run(); });
}

void HostUpload::wait(int item, hipStream_t s) {
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait(lk, [&]() { return queued_ > item || done_ || err_ != hipSuccess; });
  if (err_ != hipSuccess) throw Error(TNS_ERR_DEVICE, std::string("input upload: ") + hipGetErrorString(err_));
  if (queued_ <= item) throw Error(TNS_ERR_DEVICE, "input upload stopped early");
  lk.unlock();
  TNS_HIP(hipStreamWaitEvent(s, items_[item].ev, 0));
}

void HostUpload::wait_all(hipStream_t s) {
  for (int k = 0; k < (int)items_.size(); k++) wait(k, s);
}

}  // namespace tns
