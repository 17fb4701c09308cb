// comm.cpp -- the exchange steps of one proof sharded across ranks (one process per GPU).
//
// A sharded Twist/Shout proof exchanges only a few hundred bytes per step:
// partial G1 sums of the commitment / opening MSMs, the barycentric partial sum and node
// product of each opening, and one folded value per MLE table after the local sum-check
// rounds.  RCCL has no elliptic-curve or mod-r reduction, so every exchange is an
// allgather of the partials followed by the same (order-independent) combination on every
// rank -- all ranks then hold identical transcripts and proofs.
//
// Transports: RCCL (ncclAllGather over xGMI on the context stream, staged through a small
// device buffer), a host callback (any launcher's collective, e.g. torch.distributed), or
// the trivial one-rank communicator used by the unsharded entry points.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "common.hpp"

namespace tns {

namespace {

struct SelfComm final : Comm {
  int kind() const override { return 0; }
  void allgather(Ctx *, const void *send, size_t bytes, void *recv) override { std::memcpy(recv, send, bytes); }
};

struct CallbackComm final : Comm {
  tns_allgather_fn fn;
  void *user;
  int kind() const override { return 1; }
  void allgather(Ctx *, const void *send, size_t bytes, void *recv) override {
    const int st = fn(user, send, bytes, recv);
    if (st != 0) throw Error(TNS_ERR_DEVICE, "allgather callback failed with status " + std::to_string(st));
  }
};

#define TNS_NCCL(call)                                                                          \
  do {                                                                                          \
    ncclResult_t _r = (call);                                                                   \
    if (_r != ncclSuccess) throw Error(TNS_ERR_DEVICE, std::string("RCCL: ") + ncclGetErrorString(_r)); \
  } while (0)

struct RcclComm final : Comm {
  ncclComm_t comm = nullptr;
  DevBuf send_b, recv_b;
  // host staging owned by the communicator: the copies into and out of the collective's device
  // buffers run asynchronously from pinned memory (no pageable copy that could block on the
  // pending collective), and the caller's `recv` is written only once the stream has finished.
  // After an abort the last D2H copy may still be queued: the staging buffer stays with the
  // communicator, whose destructor waits for `done` before freeing it.
  PinnedBuf send_h, recv_h;
  hipEvent_t done = nullptr;
  ~RcclComm() override {
    if (done) {
      (void)hipEventSynchronize(done);
      (void)hipEventDestroy(done);
    }
    if (comm) (void)ncclCommDestroy(comm);
  }
  int kind() const override { return 2; }
  int seen_size() const override {
    int n = 0;
    if (!comm) throw Error(TNS_ERR_DEVICE, "RCCL communicator was aborted by an earlier timeout");
    TNS_NCCL(ncclCommCount(comm, &n));
    return n;
  }
  void allgather(Ctx *c, const void *send, size_t bytes, void *recv) override {
    if (!c) throw Error(TNS_ERR_INVALID_PARAMETERS, "the RCCL communicator needs a context");
    if (!comm) throw Error(TNS_ERR_DEVICE, "RCCL communicator was aborted by an earlier timeout");
    const size_t rb = bytes * size;
    void *ds = send_b.ensure(bytes ? bytes : 1), *dr = recv_b.ensure(rb ? rb : 1);
    void *hs = send_h.ensure(bytes ? bytes : 1), *hr = recv_h.ensure(rb ? rb : 1);
    if (!done) TNS_HIP(hipEventCreateWithFlags(&done, hipEventDisableTiming));
    std::memcpy(hs, send, bytes);
    TNS_HIP(hipMemcpyAsync(ds, hs, bytes, hipMemcpyHostToDevice, c->stream));
    TNS_NCCL(ncclAllGather(ds, dr, bytes, ncclUint8, comm, c->stream));
    TNS_HIP(hipMemcpyAsync(hr, dr, rb, hipMemcpyDeviceToHost, c->stream));
    TNS_HIP(hipEventRecord(done, c->stream));
    // wait with a deadline: a rank that never joins leaves the collective pending forever, so
    // poll the event (and RCCL's own async error) and abort the communicator past timeout_s
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned spin = 0;; spin++) {
      hipError_t q = hipEventQuery(done);
      if (q == hipSuccess) break;
      if (q != hipErrorNotReady) TNS_HIP(q);
      ncclResult_t ae = ncclSuccess;
      if (ncclCommGetAsyncError(comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
        (void)ncclCommAbort(comm);
        comm = nullptr;
        throw Error(TNS_ERR_DEVICE, std::string("RCCL allgather failed: ") + ncclGetErrorString(ae));
      }
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (el > timeout_s) {
        (void)ncclCommAbort(comm);  // releases the pending collective; the communicator is dead
        comm = nullptr;
        throw Error(TNS_ERR_DEVICE, "RCCL allgather timed out after " + std::to_string(el) +
                                        " s (a peer rank never joined; communicator aborted)");
      }
      if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    std::memcpy(recv, hr, rb);
  }
};

}  // namespace

Comm &comm_self() {
  static SelfComm self;
  return self;
}

Comm *comm_callback_new(int rank, int size, tns_allgather_fn fn, void *user) {
  if (size < 1 || rank < 0 || rank >= size || !fn) throw Error(TNS_ERR_INVALID_PARAMETERS, "bad communicator shape");
  CallbackComm *c = new CallbackComm();
  c->rank = rank;
  c->size = size;
  c->fn = fn;
  c->user = user;
  return c;
}

void comm_unique_id(uint8_t out[128]) {
  static_assert(sizeof(ncclUniqueId) <= 128, "ncclUniqueId larger than the ABI's 128 bytes");
  ncclUniqueId id;
  TNS_NCCL(ncclGetUniqueId(&id));
  std::memset(out, 0, 128);
  std::memcpy(out, &id, sizeof id);
}

Comm *comm_rccl_new(Ctx *c, int rank, int size, const uint8_t uid[128]) {
  if (size < 1 || rank < 0 || rank >= size) throw Error(TNS_ERR_INVALID_PARAMETERS, "bad communicator shape");
  RcclComm *r = new RcclComm();
  r->rank = rank;
  r->size = size;
  ncclUniqueId id;
  std::memcpy(&id, uid, sizeof id);
  TNS_HIP(hipSetDevice(c->device));
  ncclResult_t st = ncclCommInitRank(&r->comm, size, id, rank);
  if (st != ncclSuccess) {
    delete r;
    throw Error(TNS_ERR_DEVICE, std::string("RCCL init: ") + ncclGetErrorString(st));
  }
  return r;
}

void Comm::exchange(Ctx *c, const void *send, size_t bytes, void *recv, const char *what) {
  if (size == 1) {  // the shared one-rank communicator: no counters (used from many threads)
    allgather(c, send, bytes, recv);
    return;
  }
  const uint64_t step = ++seq;
  const auto t0 = std::chrono::steady_clock::now();
  try {
    allgather(c, send, bytes, recv);
  } catch (const Error &e) {
    throw Error(e.code, "rank " + std::to_string(rank) + " of " + std::to_string(size) + ": exchange #" +
                            std::to_string(step) + " (" + (what ? what : "?") + ", " + std::to_string(bytes) +
                            " B per rank): " + e.what());
  }
  const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  total_s += el;
  if (el > max_s) max_s = el;
  bytes_total += (double)bytes;
  if ((double)bytes > bytes_max) bytes_max = (double)bytes;
}

// ---------------------------------------------------------------- combined exchanges
G1Xyzz allgather_sum_g1(Ctx *c, Comm &m, const G1Xyzz &part, const char *what) {
  if (m.size == 1) return part;
  std::vector<G1Xyzz> all(m.size);
  m.exchange(c, &part, sizeof part, all.data(), what);
  G1Xyzz acc = G1Xyzz::inf();
  for (const auto &p : all) acc = xyzz_add(acc, p);
  return acc;
}

std::vector<Fr> allgather_fr(Ctx *c, Comm &m, const Fr *part, size_t k, const char *what) {
  std::vector<Fr> all(k * m.size);
  m.exchange(c, part, sizeof(Fr) * k, all.data(), what);
  return all;
}

}  // namespace tns
