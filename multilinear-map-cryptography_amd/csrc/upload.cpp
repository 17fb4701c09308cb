// upload.cpp -- host-to-device copies of the drop-in provers' inputs (tns_twist_prove /
// tns_shout_prove on the caller's pageable buffers), overlapped with the proof's first MSM.
//
// A helper thread copies the queued items in order.  A large item is split into 16 MiB chunks
// spread over kWorkers threads; each worker memcpys its chunk into one of its two pinned ring
// slots (the context's staging buffer) and DMAs it on the context's copy stream as soon as it is
// full.  tools/h2dbench.hip on the MI355X box: this sustains 52-54 GB/s of the link's 57.5
// (pinned DMA alone), where one pageable hipMemcpy of 512 MiB took 9.5-24 ms (22-56 GB/s, box-
// and run-dependent) and registering the caller's buffer in place (hipHostRegister) cost 23-26 ms
// before its DMA.  After an item's last chunk the helper records the item's event on the copy
// stream; wait() makes a stream wait for it, blocking the calling thread only until the event is
// recorded (the copies are queued), not until the bytes land.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "common.hpp"

namespace tns {

namespace {
constexpr size_t kChunk = (size_t)16 << 20;
constexpr int kWorkers = 8, kSlots = 2 * kWorkers;
constexpr size_t kDirect = (size_t)8 << 20;  // smaller items: one pageable hipMemcpyAsync
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

int HostUpload::add_narrow(uint32_t *dst32, uint64_t *dst64, const uint64_t *src, size_t n) {
  const int id = add(dst32, src, 8 * n);
  items_[id].narrow = true;
  items_[id].dst_wide = dst64;
  return id;
}

bool HostUpload::narrowed(int item) {
  std::lock_guard<std::mutex> lk(mu_);
  return items_[item].narrowed;
}

// the staging ring: kSlots chunks of pinned memory and one event per slot (its last DMA)
static char *stage_ring(Ctx *c) {
  if (!c->stage_ev[0])
    for (int s = 0; s < kSlots; s++) TNS_HIP(hipEventCreateWithFlags(&c->stage_ev[s], hipEventDisableTiming));
  return (char *)c->stage.ensure(kChunk * kSlots);
}

void HostUpload::run() {
  // runs on its own thread: nothing may escape it (std::terminate would take down a process that
  // has initialised the GPU); a failure is recorded in err_ and surfaces in wait() as a status
  try {
    run_items();
  } catch (const std::bad_alloc &) {
    std::lock_guard<std::mutex> lk(mu_);
    err_ = hipErrorOutOfMemory;
    done_ = true;
  } catch (...) {
    std::lock_guard<std::mutex> lk(mu_);
    if (err_ == hipSuccess) err_ = hipErrorUnknown;
    done_ = true;
  }
  cv_.notify_all();
}

// One transfer through the pinned ring: kWorkers threads each fill their two slots in turn and DMA
// them on the copy stream.  narrow: the source is u64 values and each chunk lands as u32 (half
// the PCIe bytes); *fits turns false if a value needs more than 32 bits (the bytes sent are then
// wrong and the caller sends the u64 array instead).
hipError_t HostUpload::transfer(char *ring, void *dst, const void *src, size_t bytes, bool narrow,
                                std::atomic<bool> *fits) {
  const size_t unit = narrow ? 8 : 1, per = narrow ? kChunk / 4 : kChunk;  // source units per chunk
  const size_t total = bytes / unit, nch = (total + per - 1) / per;
  std::vector<hipError_t> werr(kWorkers, hipSuccess);
  std::vector<std::thread> ws;
  auto body = [&](int w) {
    hipError_t e = hipSetDevice(c_->device);
    int use = 0;
    for (size_t ch = (size_t)w; ch < nch && e == hipSuccess; ch += kWorkers, use ^= 1) {
      const int slot = 2 * w + use;
      char *buf = ring + (size_t)slot * kChunk;
      const size_t off = ch * per, cnt = std::min(per, total - off);
      e = hipEventSynchronize(c_->stage_ev[slot]);  // the slot's previous DMA is done
      if (e != hipSuccess) break;
      size_t len = cnt;
      if (narrow) {
        const uint64_t *in = (const uint64_t *)src + off;
        uint32_t *o = (uint32_t *)buf;
        uint64_t any = 0;
        for (size_t i = 0; i < cnt; i++) {
          any |= in[i];
          o[i] = (uint32_t)in[i];
        }
        if (any >> 32) fits->store(false, std::memory_order_relaxed);
        len = 4 * cnt;
        e = hipMemcpyAsync((uint32_t *)dst + off, buf, len, hipMemcpyHostToDevice, c_->copy);
      } else {
        std::memcpy(buf, (const char *)src + off, len);
        e = hipMemcpyAsync((char *)dst + off, buf, len, hipMemcpyHostToDevice, c_->copy);
      }
      if (e == hipSuccess) e = hipEventRecord(c_->stage_ev[slot], c_->copy);
    }
    werr[w] = e;
  };
  try {
    for (int w = 0; w < kWorkers && (size_t)w < nch; w++) ws.emplace_back(body, w);
  } catch (...) {  // a worker that could not start: its chunks go on this thread
    for (int w = (int)ws.size(); w < kWorkers && (size_t)w < nch; w++) body(w);
  }
  for (auto &t : ws) t.join();
  for (hipError_t e : werr)
    if (e != hipSuccess) return e;
  return hipSuccess;
}

void HostUpload::run_items() {
  hipError_t err = hipSetDevice(c_->device);
  for (size_t k = 0; k < items_.size() && err == hipSuccess; k++) {
    Item &it = items_[k];
    bool narrowed = false;
    if (it.bytes < kDirect) {  // (narrow items: small arrays go over as they are)
      if (it.bytes) err = hipMemcpyAsync(it.narrow ? it.dst_wide : it.dst, it.src, it.bytes, hipMemcpyHostToDevice,
                                         c_->copy);
    } else {
      char *ring = nullptr;
      try {
        ring = stage_ring(c_);
      } catch (const Error &) {
        err = hipErrorOutOfMemory;
        break;
      }
      if (it.narrow) {
        std::atomic<bool> fits(true);
        err = transfer(ring, it.dst, it.src, it.bytes, true, &fits);
        narrowed = fits.load();
        if (err == hipSuccess && !narrowed) err = transfer(ring, it.dst_wide, it.src, it.bytes, false, nullptr);
      } else {
        err = transfer(ring, it.dst, it.src, it.bytes, false, nullptr);
      }
    }
    if (err == hipSuccess) err = hipEventRecord(it.ev, c_->copy);
    {
      std::lock_guard<std::mutex> lk(mu_);
      it.narrowed = narrowed;
      queued_ = (int)k + 1;
      if (err != hipSuccess) err_ = err;
    }
    cv_.notify_all();
  }
  std::lock_guard<std::mutex> lk(mu_);
  if (err != hipSuccess) err_ = err;
  done_ = true;
  cv_.notify_all();
}

void HostUpload::start() {
  th_ = std::thread([this]() { run(); });
}

void HostUpload::wait(int item, hipStream_t s) {
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait(lk, [&]() { return queued_ > item || done_; });
  if (err_ != hipSuccess) throw Error(TNS_ERR_DEVICE, std::string("input upload: ") + hipGetErrorString(err_));
  if (queued_ <= item) throw Error(TNS_ERR_DEVICE, "input upload stopped early");
  lk.unlock();
  TNS_HIP(hipStreamWaitEvent(s, items_[item].ev, 0));
}

void HostUpload::wait_all(hipStream_t s) {
  for (int k = 0; k < (int)items_.size(); k++) wait(k, s);
}

}  // namespace tns
