// api.hip -- the C ABI of include/tns.h and the Twist/Shout prove orchestration.
//
// Twist::prove (src/twist.rs:107-252) and Shout::prove (src/shout.rs:97-222) run with
// every bulk vector resident in HBM: one H2D of the trace, exact interpolation
// (interp.hip), two KZG commits (msm.hip), the host transcript, the sum-check fold
// chain (mle.hip), then the two openings (poly.hip synthetic division + msm.hip).
// Only commitments, 4-element round polynomials and challenges cross PCIe.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "common.hpp"

struct tns_ctx {
  tns::Ctx c;
  double timing[6] = {0, 0, 0, 0, 0, 0};
};
struct tns_srs {
  tns::Srs s;
};
struct tns_transcript {
  tns::HostTranscript t;
};
struct tns_comm {
  tns::Comm *c = nullptr;
  ~tns_comm() { delete c; }
};
struct tns_buffer {
  tns::DevBuf buf;
  size_t bytes = 0;
  int device = 0;
};

namespace tns {

static thread_local std::string g_last_error;
void set_last_error(const std::string &m) { g_last_error = m; }

Ctx::~Ctx() {
  for (auto *p : plans) delete p;
  for (auto &kv : pass_tw) delete kv.second;
  for (auto &kv : bary_w) delete kv.second;
  if (lanes[1].stream) (void)hipStreamDestroy(lanes[1].stream);
  if (side) (void)hipStreamDestroy(side);
  if (copy) (void)hipStreamDestroy(copy);
  if (acc) (void)hipStreamDestroy(acc);
  for (hipEvent_t e : stage_ev)
    if (e) (void)hipEventDestroy(e);
  if (stream) (void)hipStreamDestroy(stream);
}

template <class F>
static int guarded(F &&f) {
  try {
    return f();
  } catch (const Error &e) {
    set_last_error(e.what());
    return e.code;
  } catch (const std::exception &e) {
    set_last_error(e.what());
    return TNS_ERR_DEVICE;
  }
}

static void store_proj(const G1Affine &a, uint64_t out[12]) {
  G1Jac j = affine_to_jac(a);
  std::memcpy(out, &j, sizeof j);
}
static G1Affine proj_to_affine_host(const uint64_t in[12]) {
  G1Jac j;
  std::memcpy(&j, in, sizeof j);
  G1Affine a;
  if (j.z.is_zero()) {
    a.x = Fq::zero();
    a.y = Fq::zero();
    return a;
  }
  Fq zi = inv(j.z), zi2 = sqr(zi);
  a.x = mul(j.x, zi2);
  a.y = mul(j.y, mul(zi2, zi));
  return a;
}

struct Timer {
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  double ms() const {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
};

// KZGCommitment::commit on device-resident coefficients (src/commitments.rs:162-180)
static G1Affine commit_dev(Ctx *c, const Srs &srs, const Fr *coeffs, size_t n) {
  if (n > srs.n) throw Error(TNS_ERR_COMMITMENT, "Polynomial degree exceeds setup size");
  if (srs.first != 0 || srs.held < n)
    throw Error(TNS_ERR_INVALID_PARAMETERS, "coefficient commitments need the whole SRS (this is a shard)");
  return xyzz_to_affine(msm_dev(c, srs.points.as<G1Affine>(), coeffs, n, srs_fixed_base(c, srs, n)));
}

// KZGCommitment::open on device-resident coefficients (src/commitments.rs:182-199)
static void open_dev(Ctx *c, const Srs &srs, const Fr *coeffs, size_t n, const Fr &z, Fr *value,
                     G1Affine *proof, DevBuf &sbuf) {
  if (n == 0) {
    *value = Fr::zero();
    proof->x = Fq::zero();
    proof->y = Fq::zero();
    return;
  }
  Fr *s = (Fr *)sbuf.ensure(sizeof(Fr) * n);
  *value = synthetic_division_dev(c, coeffs, n, z, s);
  // quotient q_i = s_{i+1}, length n - 1 (empty for n == 1 -> identity)
  *proof = commit_dev(c, srs, s + 1, n - 1);
}

// One committed vector of Twist/Shout::prove: evaluations y on the nodes 0..N-1
// (vector_to_polynomial input, src/polynomials.rs:248-262), of which this rank holds the
// slice [first, first + cnt).  Committed and opened via the Lagrange basis when the SRS
// provides it (partial MSMs summed over the ranks), else via interpolated coefficients.
struct EvalPoly {
  const Fr *y = nullptr;       // device, cnt (must stay intact until opened)
  Fr *coeffs = nullptr;        // device scratch, N (coefficient path, unsharded only)
  size_t N = 0, first = 0, cnt = 0;
  const LagrangeBasis *basis = nullptr;
  bool have_coeffs = false;
};

static G1Affine commit_evals(Ctx *c, const Srs &srs, EvalPoly &p, Comm &m) {
  if (p.N > srs.n) throw Error(TNS_ERR_COMMITMENT, "Polynomial degree exceeds setup size");
  p.basis = lagrange_basis_dev(c, srs, p.N, p.first, p.cnt);
  if (p.basis) {
    const G1Xyzz part = msm_dev(c, p.basis->points.as<G1Affine>(), p.y, p.cnt, p.basis->fb);
    return xyzz_to_affine(allgather_sum_g1(c, m, part, "commitment partial MSM"));
  }
  if (m.size > 1) throw Error(TNS_ERR_INVALID_PARAMETERS, "sharded proving needs an SRS with tau (Lagrange basis)");
  if (p.N & (p.N - 1))
    throw Error(TNS_ERR_POLYNOMIAL, "interpolation of a non-power-of-two vector needs an SRS with tau (Lagrange basis)");
  interpolate_consecutive_dev(c, p.y, p.N, p.coeffs);
  p.have_coeffs = true;
  return commit_dev(c, srs, p.coeffs, p.N);
}

static void open_evals(Ctx *c, const Srs &srs, EvalPoly &p, const Fr &z, Fr *value, G1Affine *proof,
                       DevBuf &sbuf, Comm &m) {
  if (p.basis && m.size == 1 && fr_is_node(z, p.N)) {  // z = j0 is a node: value y_j0, derivative term
    const size_t j0 = (size_t)from_mont(z).v[0];
    Fr *q = (Fr *)sbuf.ensure(sizeof(Fr) * p.N);
    TNS_HIP(hipMemcpyAsync(value, p.y + j0, sizeof(Fr), hipMemcpyDeviceToHost, c->stream));
    lagrange_node_quotient_dev(c, p.y, p.N, j0, q);  // synchronises
    *proof = xyzz_to_affine(msm_dev(c, p.basis->points.as<G1Affine>(), q, p.N, p.basis->fb));
    return;
  }
  if (p.basis && !fr_is_node(z, p.N)) {
    Fr *q = (Fr *)sbuf.ensure(sizeof(Fr) * p.cnt);
    Fr part[2];
    lagrange_open_partial_dev(c, p.y, p.N, p.first, p.cnt, z, q, &part[0], &part[1]);
    Fr ell = Fr::one(), S = Fr::zero();
    if (m.size == 1) {
      ell = part[0];
      S = part[1];
    } else {
      const std::vector<Fr> all = allgather_fr(c, m, part, 2, "barycentric partials");
      for (int r = 0; r < m.size; r++) {
        ell = mul(ell, all[2 * r]);
        S = add(S, all[2 * r + 1]);
      }
    }
    *value = mul(ell, S);  // P(z) = ell(z) sum_j w_j y_j / (z - j)
    lagrange_quotient_finish_dev(c, p.y, p.cnt, *value, q);
    const G1Xyzz pp = msm_dev(c, p.basis->points.as<G1Affine>(), q, p.cnt, p.basis->fb);
    *proof = xyzz_to_affine(allgather_sum_g1(c, m, pp, "opening partial MSM"));
    return;
  }
  if (m.size > 1)  // z on a node: probability ~2^-230; the coefficient route is unsharded
    throw Error(TNS_ERR_PROOF_GENERATION, "opening challenge is an interpolation node (sharded prover)");
  if (!p.have_coeffs) {  // no basis: coefficient form
    if (p.N & (p.N - 1))
      throw Error(TNS_ERR_POLYNOMIAL, "interpolation of a non-power-of-two vector needs an SRS with tau (Lagrange basis)");
    interpolate_consecutive_dev(c, p.y, p.N, p.coeffs);
    p.have_coeffs = true;
  }
  open_dev(c, srs, p.coeffs, p.N, z, value, proof, sbuf);
}

// Both vectors of a proof at once (the two commitments; the two openings at the same z):
// their MSMs overlap on the context's two lanes and each exchange step carries both.
static G1Xyzz sum_rank_parts(const G1Xyzz *all, int size, int stride, int k) {
  G1Xyzz acc = G1Xyzz::inf();
  for (int r = 0; r < size; r++) acc = xyzz_add(acc, all[(size_t)r * stride + k]);
  return acc;
}

// What rides along with an exchange of MSM partials (the exchanges of a sharded proof are few and
// latency-bound, so independent payloads share one): `bytes` of this rank's data, every rank's
// copy landing rank-major in `all` (size * bytes).
struct ExtraPayload {
  const void *data = nullptr;
  size_t bytes = 0;  // a multiple of 4
  std::vector<uint8_t> all;
};

static void allgather_sum_g1_pair(Ctx *c, Comm &m, const G1Xyzz part[2], G1Affine out[2], const char *what,
                                  ExtraPayload *extra = nullptr) {
  const size_t xb = extra ? extra->bytes : 0;
  if (m.size == 1) {
    xyzz_to_affine2(part[0], part[1], out[0], out[1]);
    if (xb) extra->all.assign((const uint8_t *)extra->data, (const uint8_t *)extra->data + xb);
    return;
  }
  // one message per rank: [partial 0 | partial 1 | extra], G1Xyzz-aligned
  const size_t rec = 2 * sizeof(G1Xyzz) + (xb + sizeof(G1Xyzz) - 1) / sizeof(G1Xyzz) * sizeof(G1Xyzz);
  const size_t recw = rec / sizeof(G1Xyzz);
  std::vector<G1Xyzz> mine(recw), all(recw * (size_t)m.size);
  mine[0] = part[0];
  mine[1] = part[1];
  if (xb) std::memcpy(&mine[2], extra->data, xb);
  m.exchange(c, mine.data(), rec, all.data(), what);
  xyzz_to_affine2(sum_rank_parts(all.data(), m.size, (int)recw, 0), sum_rank_parts(all.data(), m.size, (int)recw, 1),
                  out[0], out[1]);
  if (xb) {
    extra->all.resize(xb * (size_t)m.size);
    for (int r = 0; r < m.size; r++)
      std::memcpy(extra->all.data() + xb * (size_t)r, &all[recw * (size_t)r + 2], xb);
  }
}

// src0 / src1 (optional): how p0.y / p1.y get written (on the MSM lane that reads them)
// extra (optional, sharded): data exchanged with the commitments' partial sums
static void commit_evals_pair(Ctx *c, const Srs &srs, EvalPoly &p0, EvalPoly &p1, Comm &m, G1Affine out[2],
                              const ScalarSource *src0 = nullptr, const ScalarSource *src1 = nullptr,
                              ExtraPayload *extra = nullptr) {
  if (p0.N > srs.n || p1.N > srs.n) throw Error(TNS_ERR_COMMITMENT, "Polynomial degree exceeds setup size");
  p0.basis = lagrange_basis_dev(c, srs, p0.N, p0.first, p0.cnt);
  p1.basis = lagrange_basis_dev(c, srs, p1.N, p1.first, p1.cnt);
  if (!p0.basis || !p1.basis) {
    for (const ScalarSource *s : {src0, src1})
      if (s && s->prep) s->prep(c->stream);
    if (extra && extra->bytes && m.size > 1)  // (the coefficient route is unsharded: never taken here)
      throw Error(TNS_ERR_PROOF_GENERATION, "sharded commitment without a Lagrange basis");
    if (extra) extra->all.assign((const uint8_t *)extra->data, (const uint8_t *)extra->data + extra->bytes);
    out[0] = commit_evals(c, srs, p0, m);
    out[1] = commit_evals(c, srs, p1, m);
    return;
  }
  auto args = [](const EvalPoly &p, const ScalarSource *s) {
    MsmArgs a{p.basis->points.as<G1Affine>(), p.y, p.cnt, p.basis->fb};
    if (s) {
      a.prep = s->prep;
      a.late = s->late;
      a.chunks = s->chunks;
      a.chunk_off = s->chunk_off;
      a.chunk_prep = s->chunk_prep;
      a.canon = s->canon;
      a.canon_bits = s->canon_bits;
      a.u64 = s->u64;
      a.n_u64 = s->n_u64;
    }
    return a;
  };
  G1Xyzz part[2];
  msm_pair_dev(c, args(p0, src0), args(p1, src1), part);
  allgather_sum_g1_pair(c, m, part, out, "commitment pair partial MSMs", extra);
}

// extra (optional): exchanged with the openings' partial sums once extra_ready() has run (the
// sharded sum-check's folded table values, which the side stream computes under the openings)
// side_work (optional): host work to queue once the barycentric pass is on the device (it runs
// before the pass's first host wait instead of in front of its launches)
static void open_evals_pair(Ctx *c, const Srs &srs, EvalPoly &p0, EvalPoly &p1, const Fr &z, Fr value[2],
                            G1Affine proof[2], DevBuf &sbuf0, DevBuf &sbuf1, Comm &m,
                            ExtraPayload *extra = nullptr, const std::function<void()> &extra_ready = nullptr,
                            const std::function<void()> &side_work = nullptr) {
  const bool same_nodes = p0.N == p1.N && p0.first == p1.first && p0.cnt == p1.cnt;
  const bool pair_pass = p0.basis && p1.basis && !fr_is_node(z, p0.N) && !fr_is_node(z, p1.N) && same_nodes;
  if (side_work && !pair_pass) side_work();
  if (!p0.basis || !p1.basis || fr_is_node(z, p0.N) || fr_is_node(z, p1.N)) {
    open_evals(c, srs, p0, z, &value[0], &proof[0], sbuf0, m);
    open_evals(c, srs, p1, z, &value[1], &proof[1], sbuf0, m);
    if (extra) {  // (unsharded here: open_evals refuses a node z with several ranks)
      if (extra_ready) extra_ready();
      extra->all.assign((const uint8_t *)extra->data, (const uint8_t *)extra->data + extra->bytes);
    }
    return;
  }
  Fr *q0 = (Fr *)sbuf0.ensure(sizeof(Fr) * p0.cnt), *q1 = (Fr *)sbuf1.ensure(sizeof(Fr) * p1.cnt);
  Fr part[4];
  // the shared-inverse pass hands the MSMs canonical quotients and their bit lengths; its
  // inverses come out canonical too, so the quotient kernel needs no reduction pass
  // (0.540 -> 0.504 ms at C4, profiles/r04_c4_step_timeline_canon_inv.txt)
  const bool canon_q = same_nodes && p0.cnt > 64, canon_inv = canon_q;
  if (same_nodes) {  // Twist: one batch inversion for both vectors (inverses land in q1)
    Fr p3[3];
    lagrange_open_partial2_dev(c, p0.y, p1.y, p0.N, p0.first, p0.cnt, z, q1, p3, canon_inv, side_work);
    part[0] = part[2] = p3[0];
    part[1] = p3[1];
    part[3] = p3[2];
  } else {
    lagrange_open_partial_dev(c, p0.y, p0.N, p0.first, p0.cnt, z, q0, &part[0], &part[1]);
    lagrange_open_partial_dev(c, p1.y, p1.N, p1.first, p1.cnt, z, q1, &part[2], &part[3]);
  }
  Fr ell[2] = {Fr::one(), Fr::one()}, S[2] = {Fr::zero(), Fr::zero()};
  const std::vector<Fr> all = allgather_fr(c, m, part, 4, "barycentric pair partials");
  for (int r = 0; r < m.size; r++)
    for (int k = 0; k < 2; k++) {
      ell[k] = mul(ell[k], all[4 * (size_t)r + 2 * k]);
      S[k] = add(S[k], all[4 * (size_t)r + 2 * k + 1]);
    }
  for (int k = 0; k < 2; k++) value[k] = mul(ell[k], S[k]);  // P(z) = ell(z) sum_j w_j y_j / (z - j)
  unsigned *qbits = canon_q ? (unsigned *)c->qbits.ensure(2 * sizeof(unsigned)) : nullptr;
  // the shared-table plan both opening MSMs will take (full-width quotients): the quotient kernel
  // also counts pass 1 of both bucket sorts (their count kernels and one read of q0 / q1 go)
  const FixedBase *f0 = p0.basis->fb, *f1 = p1.basis->fb;
  const uint32_t *pre[2] = {nullptr, nullptr};
  bool fused = false;
  if (same_nodes && canon_inv && c->msm_tables && f0 && f1 && f0->c == f1->c && f0->W == f1->W)
    fused = quotient2_count_dev(c, p0.y, p1.y, p0.cnt, value[0], value[1], q1, q0, q1, qbits, f0->c, f0->W, pre);
  if (fused) {
  } else if (same_nodes) {
    lagrange_quotient_finish2_dev(c, p0.y, p1.y, p0.cnt, value[0], value[1], q1, q0, q1, qbits, canon_inv);
  } else {
    lagrange_quotient_finish_dev(c, p0.y, p0.cnt, value[0], q0);
    lagrange_quotient_finish_dev(c, p1.y, p1.cnt, value[1], q1);
  }
  G1Xyzz pp[2];
  MsmArgs a0{p0.basis->points.as<G1Affine>(), q0, p0.cnt, p0.basis->fb, qbits};
  MsmArgs a1{p1.basis->points.as<G1Affine>(), q1, p1.cnt, p1.basis->fb, qbits ? qbits + 1 : nullptr};
  if (fused) {  // (lane 0 sorts a0, lane 1 a1: neither is late)
    a0.precounted = pre[0];
    a1.precounted = pre[1];
    a0.pre_c = a1.pre_c = f0->c;
    a0.pre_W = a1.pre_W = f0->W;
    a0.plan_bits = a1.plan_bits = 254;  // (the counts assumed the full-width table plan)
  }
  msm_pair_dev(c, a0, a1, pp);
  if (extra && extra_ready) extra_ready();
  allgather_sum_g1_pair(c, m, pp, proof, extra ? "opening pair partial MSMs + folded table values" : "opening pair partial MSMs",
                        extra);
}

// shard geometry: `size` ranks over N padded entries (size a power of two <= N)
static void check_shard(const Comm &m, size_t N, const char *what) {
  if (m.size & (m.size - 1)) throw Error(TNS_ERR_INVALID_PARAMETERS, "rank count must be a power of two");
  if ((size_t)m.size > N)
    throw Error(TNS_ERR_INVALID_PARAMETERS, std::string("more ranks than padded ") + what + " entries");
}
static size_t slice_count(uint64_t n_total, size_t first, size_t L) {
  return n_total <= first ? 0 : (size_t)std::min<uint64_t>(L, n_total - first);
}

// multi-threaded element-wise host conversion
template <class C, class F>
static void par_convert(const uint64_t *in, size_t n, uint64_t *out, F f) {
  unsigned nt = std::thread::hardware_concurrency();
  if (nt < 1) nt = 1;
  if (nt > 16) nt = 16;
  if (n < 4096) nt = 1;
  std::vector<std::thread> th;
  size_t per = (n + nt - 1) / nt;
  for (unsigned t = 0; t < nt; t++) {
    size_t a = t * per, b = std::min(n, a + per);
    if (a >= b) break;
    th.emplace_back([=]() {
      for (size_t i = a; i < b; i++) f(in, out, i);
    });
  }
  for (auto &x : th) x.join();
}

}  // namespace tns

using namespace tns;

extern "C" {

const char *tns_last_error(void) { return g_last_error.c_str(); }
int tns_version(void) { return 100; }
int tns_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int tns_device_info_get(int device, tns_device_info *out) {
  return guarded([&]() {
    if (!out) throw Error(TNS_ERR_INVALID_PARAMETERS, "null output");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
      throw Error(TNS_ERR_NO_DEVICE, "no HIP device visible");
    if (device < 0 || device >= n) throw Error(TNS_ERR_INVALID_PARAMETERS, "device index out of range");
    hipDeviceProp_t p;
    TNS_HIP(hipGetDeviceProperties(&p, device));
    std::memset(out, 0, sizeof(*out));
    std::snprintf(out->name, sizeof(out->name), "%s", p.name);
    std::snprintf(out->arch, sizeof(out->arch), "%s", p.gcnArchName);
    std::snprintf(out->pci_bus_id, sizeof(out->pci_bus_id), "%04x:%02x:%02x.0", p.pciDomainID, p.pciBusID,
                  p.pciDeviceID);
    out->clock_khz = p.clockRate;
    out->mem_clock_khz = p.memoryClockRate;
    out->cu_count = p.multiProcessorCount;
    out->total_mem = p.totalGlobalMem;
    return TNS_OK;
  });
}

// The context's five streams.  Created in this order: with GPU_MAX_HW_QUEUES = 4 (HIP's default)
// the fifth stream shares the first one's hardware queue, and the copy stream (drop-in uploads,
// during the commitments) and the accumulation stream (only in the openings of a drop-in proof)
// are never busy together -- the copy stream on the context stream's queue serialised the upload
// behind the commitments (+1.4 ms per drop-in C4 step, profiles/r06_ab_stream_priority.txt).
// prio: the accumulations at the least priority and the context stream (lane 0) at the greatest,
// lane 1 / side / copy normal -- lane 1's last sort passes then wait for the first accumulation's
// tail-off instead of running beside it (-0.3-0.45 ms per C4 step); off for processes sharing a
// GPU, whose least-priority queues starve behind the other processes' (TNS_CTX_NO_STREAM_PRIORITIES;
// chosen at creation: streams recreated without priorities in the same process kept the pathology).
static void create_streams(Ctx &c, bool prio) {
  int lo = 0, hi = 0;
  TNS_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
  if (!prio) lo = hi = 0;
  auto mk = [](hipStream_t *s, int p) {
    TNS_HIP(p ? hipStreamCreateWithPriority(s, hipStreamNonBlocking, p) : hipStreamCreateWithFlags(s, hipStreamNonBlocking));
  };
  mk(&c.acc, lo);
  mk(&c.stream, hi);
  c.lanes[0].stream = c.stream;
  mk(&c.lanes[1].stream, 0);
  mk(&c.side, 0);
  mk(&c.copy, 0);
}

int tns_ctx_create(int device, tns_ctx **out) { return tns_ctx_create_ex(device, 0, out); }

int tns_ctx_create_ex(int device, unsigned flags, tns_ctx **out) {
  return guarded([&]() {
    if (flags & ~TNS_CTX_NO_STREAM_PRIORITIES) throw Error(TNS_ERR_INVALID_PARAMETERS, "unknown context flags");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
      throw Error(TNS_ERR_NO_DEVICE, "no HIP device visible");
    if (device < 0 || device >= n) throw Error(TNS_ERR_INVALID_PARAMETERS, "device index out of range");
    TNS_HIP(hipSetDevice(device));
    hipDeviceProp_t prop;
    TNS_HIP(hipGetDeviceProperties(&prop, device));
    if (std::string(prop.gcnArchName).rfind("gfx950", 0) != 0)
      throw Error(TNS_ERR_NO_DEVICE, std::string("libtns is built for gfx950, device is ") + prop.gcnArchName);
    tns_ctx *x = new tns_ctx();
    x->c.device = device;
    x->c.num_cu = prop.multiProcessorCount;
    try {
      create_streams(x->c, !(flags & TNS_CTX_NO_STREAM_PRIORITIES));
    } catch (...) {
      delete x;
      throw;
    }
    *out = x;
    return TNS_OK;
  });
}

void tns_ctx_destroy(tns_ctx *ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->c.device);
  (void)hipStreamSynchronize(ctx->c.stream);
  if (ctx->c.side) (void)hipStreamSynchronize(ctx->c.side);
  if (ctx->c.acc) (void)hipStreamSynchronize(ctx->c.acc);
  delete ctx;
}

int tns_ctx_synchronize(tns_ctx *ctx) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    TNS_HIP(hipStreamSynchronize(ctx->c.stream));
    return TNS_OK;
  });
}

// setup_params (src/utils.rs:79-131) for ranks [rank] of [size]: the SRS holds the
// contiguous share [first, first + held) of the num_powers g1_powers (all of them for size 1)
static void setup_core(tns_ctx *ctx, unsigned log_size, int rank, int size, tns_params *out, tns_srs **srs_out) {
  if (log_size > 26) throw Error(TNS_ERR_INVALID_PARAMETERS, "log_size too large");
  if (size < 1 || rank < 0 || rank >= size) throw Error(TNS_ERR_INVALID_PARAMETERS, "bad shard");
  std::memset(out, 0, sizeof *out);
  out->log_size = log_size;
  out->max_operations = (uint64_t)1 << (log_size + 2);  // src/utils.rs:80
  out->num_powers = next_pow2(out->max_operations) + 1;  // src/utils.rs:89
  uint8_t seed42[32];
  std::memset(seed42, 42, 32);
  Fr tau = host_fr_rand_chacha(seed42, out->fiat_shamir_seed);  // src/utils.rs:81-84, 101-102
  std::memcpy(out->tau, &tau, 32);
  if (!srs_out) return;
  *srs_out = nullptr;
  CtxScope g(&ctx->c);
  tns_srs *s = new tns_srs();
  s->s.device = ctx->c.device;
  s->s.n = out->num_powers;
  // shares of the 2^k + 1 powers: [r 2^k/size, (r + 1) 2^k/size), the last rank also holding
  // g1_powers[2^k] -- so rank r's share covers the coefficient slice of tns_shard_slice
  // (tns_msm_sharded); any other count splits as evenly as possible
  const size_t m = s->s.n - 1;
  if (m % (size_t)size == 0 && m >= (size_t)size) {
    s->s.first = (size_t)rank * (m / size);
    s->s.held = m / size + (rank == size - 1 ? 1 : 0);
  } else {
    const size_t base = s->s.n / size, rem = s->s.n % size;
    s->s.first = (size_t)rank * base + std::min<size_t>(rank, rem);
    s->s.held = base + ((size_t)rank < rem ? 1 : 0);
  }
  s->s.has_tau = true;
  s->s.tau = tau;
  try {
    G1Affine *pts = (G1Affine *)s->s.points.ensure(sizeof(G1Affine) * (s->s.held ? s->s.held : 1));
    srs_generate_dev(&ctx->c, tau, s->s.first, s->s.held, pts);
  } catch (...) {
    delete s;
    throw;
  }
  *srs_out = s;
}

int tns_setup_params(tns_ctx *ctx, unsigned log_size, tns_params *out, tns_srs **srs_out) {
  return guarded([&]() {
    setup_core(ctx, log_size, 0, 1, out, srs_out);
    return TNS_OK;
  });
}

int tns_setup_params_shard(tns_ctx *ctx, unsigned log_size, int rank, int size, tns_params *out,
                           tns_srs **srs_out) {
  return guarded([&]() {
    setup_core(ctx, log_size, rank, size, out, srs_out);
    return TNS_OK;
  });
}

int tns_srs_upload(tns_ctx *ctx, const uint64_t *g1, size_t n, tns_srs **out) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    tns_srs *s = new tns_srs();
    s->s.device = ctx->c.device;
    s->s.n = n;
    s->s.held = n;
    try {
      void *p = s->s.points.ensure(sizeof(G1Affine) * (n ? n : 1));
      if (n) TNS_HIP(hipMemcpy(p, g1, sizeof(G1Affine) * n, hipMemcpyHostToDevice));
    } catch (...) {
      delete s;
      throw;
    }
    *out = s;
    return TNS_OK;
  });
}

int tns_srs_download(tns_ctx *ctx, const tns_srs *srs, uint64_t *g1_out, size_t n) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    if (srs->s.first != 0 || n > srs->s.held) throw Error(TNS_ERR_INVALID_PARAMETERS, "download beyond SRS length");
    if (n) TNS_HIP(hipMemcpy(g1_out, srs->s.points.p, sizeof(G1Affine) * n, hipMemcpyDeviceToHost));
    return TNS_OK;
  });
}

int tns_srs_download_indices(tns_ctx *ctx, const tns_srs *srs, const uint64_t *idx, size_t k,
                             uint64_t *g1_out) {
  return guarded([&]() {
    if (!ctx || !srs) throw Error(TNS_ERR_INVALID_PARAMETERS, "null context or SRS");
    if (k > 0 && (!idx || !g1_out)) throw Error(TNS_ERR_INVALID_PARAMETERS, "null index or output buffer");
    CtxScope g(&ctx->c);
    for (size_t t = 0; t < k; t++)
      if (idx[t] < srs->s.first || idx[t] >= srs->s.first + srs->s.held)
        throw Error(TNS_ERR_INVALID_PARAMETERS, "SRS index outside this SRS's share");
    const G1Affine *pts = srs->s.points.as<G1Affine>();
    for (size_t t = 0; t < k; t++)
      TNS_HIP(hipMemcpyAsync(g1_out + 8 * t, pts + (idx[t] - srs->s.first), sizeof(G1Affine), hipMemcpyDeviceToHost,
                             ctx->c.stream));
    TNS_HIP(hipStreamSynchronize(ctx->c.stream));
    return TNS_OK;
  });
}

int tns_srs_share(const tns_srs *srs, uint64_t *first, uint64_t *held) {
  return guarded([&]() {
    if (!srs || !first || !held) throw Error(TNS_ERR_INVALID_PARAMETERS, "null SRS or output");
    *first = srs->s.first;
    *held = srs->s.held;
    return TNS_OK;
  });
}

size_t tns_srs_len(const tns_srs *srs) { return srs ? srs->s.n : 0; }

int tns_srs_set_tau(tns_srs *srs, const uint64_t tau[4]) {
  return guarded([&]() {
    if (!srs) throw Error(TNS_ERR_INVALID_PARAMETERS, "null SRS");
    Fr t;
    std::memcpy(&t, tau, 32);
    // The Lagrange basis (every commitment and opening of the Lagrange route) is derived from
    // tau, so tau must be the trapdoor of the uploaded powers: one held point g1_powers[e]
    // (e = 1, or the shard's first index) is checked against tau^e * G1 on the host.  An SRS
    // holding no such point (only g1_powers[0] = G1) cannot contradict tau.
    const size_t e = srs->s.first ? srs->s.first : 1;
    if (e >= srs->s.first && e < srs->s.first + srs->s.held) {
      TNS_HIP(hipSetDevice(srs->s.device));
      G1Affine held;
      TNS_HIP(hipMemcpy(&held, srs->s.points.as<G1Affine>() + (e - srs->s.first), sizeof(G1Affine),
                        hipMemcpyDeviceToHost));
      const G1Affine want = xyzz_to_affine(g1_mul_host(g1_generator_host(), pow_u64(t, (u64)e)));
      if (!(held.x == want.x) || !(held.y == want.y))
        throw Error(TNS_ERR_INVALID_PARAMETERS, "tau does not match the SRS (g1_powers[e] != tau^e * G1)");
    }
    for (auto &kv : srs->s.lagrange) delete kv.second;
    srs->s.lagrange.clear();
    srs->s.tau = t;
    srs->s.has_tau = true;
    return TNS_OK;
  });
}

int tns_srs_prepare_lagrange(tns_ctx *ctx, tns_srs *srs, size_t n) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    if (!srs->s.has_tau) throw Error(TNS_ERR_INVALID_PARAMETERS, "SRS has no tau");
    if (n == 0 || (n & (n - 1))) throw Error(TNS_ERR_INVALID_PARAMETERS, "Lagrange basis size must be a power of two");
    const bool saved = ctx->c.lagrange_commit;
    ctx->c.lagrange_commit = true;
    const LagrangeBasis *b = lagrange_basis_dev(&ctx->c, srs->s, n, 0, n);
    ctx->c.lagrange_commit = saved;
    (void)b;  // nullptr only when tau is itself a node: the coefficient path is used then
    return TNS_OK;
  });
}

int tns_srs_prepare_lagrange_from_powers(tns_ctx *ctx, tns_srs *srs, size_t n) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    (void)lagrange_basis_from_powers_dev(&ctx->c, srs->s, n);
    return TNS_OK;
  });
}

int tns_srs_lagrange_download(tns_ctx *ctx, tns_srs *srs, size_t n, uint64_t *g1_affine_out) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    if (!srs->s.has_tau && !srs->s.lagrange.count(std::make_tuple(n, (size_t)0, n)))
      throw Error(TNS_ERR_INVALID_PARAMETERS, "SRS has no tau (and no basis prepared from its powers)");
    if (n == 0 || (n & (n - 1))) throw Error(TNS_ERR_INVALID_PARAMETERS, "Lagrange basis size must be a power of two");
    const bool saved = ctx->c.lagrange_commit;
    ctx->c.lagrange_commit = true;
    const LagrangeBasis *b = lagrange_basis_dev(&ctx->c, srs->s, n, 0, n);
    ctx->c.lagrange_commit = saved;
    if (!b) throw Error(TNS_ERR_INVALID_PARAMETERS, "tau is an interpolation node: no Lagrange basis");
    TNS_HIP(hipMemcpy(g1_affine_out, b->points.p, sizeof(G1Affine) * n, hipMemcpyDeviceToHost));
    return TNS_OK;
  });
}

int tns_ctx_set_msm_tables(tns_ctx *ctx, int on) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    ctx->c.msm_tables = on != 0;
    return TNS_OK;
  });
}

int tns_ctx_set_upload_chunks(tns_ctx *ctx, int chunks) {
  return guarded([&]() {
    if (!ctx) throw Error(TNS_ERR_INVALID_PARAMETERS, "null context");
    if (chunks < 1 || chunks > 64) throw Error(TNS_ERR_INVALID_PARAMETERS, "upload chunks must be 1..64");
    CtxScope g(&ctx->c);
    ctx->c.upload_chunks = chunks;
    return TNS_OK;
  });
}

int tns_ctx_set_commit_basis(tns_ctx *ctx, int lagrange) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    ctx->c.lagrange_commit = lagrange != 0;
    return TNS_OK;
  });
}
void tns_srs_destroy(tns_srs *srs) {
  if (!srs) return;
  (void)hipSetDevice(srs->s.device);
  delete srs;
}

int tns_kzg_commit(tns_ctx *ctx, const tns_srs *srs, const uint64_t *coeffs, size_t n, uint64_t out[12]) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    if (n > srs->s.n) throw Error(TNS_ERR_COMMITMENT, "Polynomial degree exceeds setup size");
    DevBuf d;
    Fr *dc = (Fr *)d.ensure(sizeof(Fr) * (n ? n : 1));
    if (n) TNS_HIP(hipMemcpyAsync(dc, coeffs, sizeof(Fr) * n, hipMemcpyHostToDevice, ctx->c.stream));
    store_proj(commit_dev(&ctx->c, srs->s, dc, n), out);
    return TNS_OK;
  });
}

static void upload_evals(tns_ctx *ctx, const uint64_t *evals, size_t n, DevBuf &d, DevBuf &cf, EvalPoly &p) {
  if (n == 0) throw Error(TNS_ERR_POLYNOMIAL, "empty evaluation vector");
  Fr *dy = (Fr *)d.ensure(sizeof(Fr) * n);
  TNS_HIP(hipMemcpyAsync(dy, evals, sizeof(Fr) * n, hipMemcpyHostToDevice, ctx->c.stream));
  p.y = dy;
  p.N = n;
  p.first = 0;
  p.cnt = n;
  p.coeffs = (Fr *)cf.ensure(sizeof(Fr) * n);
}

int tns_kzg_commit_evals(tns_ctx *ctx, const tns_srs *srs, const uint64_t *evals, size_t n, uint64_t out[12]) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    DevBuf d, cf;
    EvalPoly p;
    upload_evals(ctx, evals, n, d, cf, p);
    store_proj(commit_evals(&ctx->c, srs->s, p, comm_self()), out);
    return TNS_OK;
  });
}

int tns_kzg_open_evals(tns_ctx *ctx, const tns_srs *srs, const uint64_t *evals, size_t n, const uint64_t z[4],
                       uint64_t value[4], uint64_t proof[12]) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    DevBuf d, cf, s;
    EvalPoly p;
    upload_evals(ctx, evals, n, d, cf, p);
    if (n > srs->s.n) throw Error(TNS_ERR_COMMITMENT, "Polynomial degree exceeds setup size");
    p.basis = lagrange_basis_dev(&ctx->c, srs->s, n, 0, n);
    Fr zz, v;
    std::memcpy(&zz, z, 32);
    G1Affine pi;
    open_evals(&ctx->c, srs->s, p, zz, &v, &pi, s, comm_self());
    std::memcpy(value, &v, 32);
    store_proj(pi, proof);
    return TNS_OK;
  });
}

// KZGVectorCommitment (src/commitments.rs:408-483): commit = commit(interpolant of v on
// 0..n-1), any n; open at index i = KZG open at the node i (value v_i).
int tns_vc_open(tns_ctx *ctx, const tns_srs *srs, const uint64_t *vec, size_t n, size_t index, uint64_t value[4],
                uint64_t proof[12]) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    if (index >= n) throw Error(TNS_ERR_COMMITMENT, "Index out of bounds");
    DevBuf d, cf, s;
    EvalPoly p;
    upload_evals(ctx, vec, n, d, cf, p);
    if (n > srs->s.n) throw Error(TNS_ERR_COMMITMENT, "Polynomial degree exceeds setup size");
    p.basis = lagrange_basis_dev(&ctx->c, srs->s, n, 0, n);
    const Fr z = from_u64<FrCfg>((uint64_t)index);
    Fr v;
    G1Affine pi;
    open_evals(&ctx->c, srs->s, p, z, &v, &pi, s, comm_self());
    std::memcpy(value, &v, 32);
    store_proj(pi, proof);
    return TNS_OK;
  });
}

int tns_msm(tns_ctx *ctx, const tns_srs *srs, const uint64_t *scalars, size_t n, uint64_t out[12]) {
  return tns_kzg_commit(ctx, srs, scalars, n, out);
}

int tns_kzg_open(tns_ctx *ctx, const tns_srs *srs, const uint64_t *coeffs, size_t n, const uint64_t z[4],
                 uint64_t value[4], uint64_t proof[12]) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    DevBuf d, s;
    Fr *dc = (Fr *)d.ensure(sizeof(Fr) * (n ? n : 1));
    if (n) TNS_HIP(hipMemcpyAsync(dc, coeffs, sizeof(Fr) * n, hipMemcpyHostToDevice, ctx->c.stream));
    Fr zz, v;
    std::memcpy(&zz, z, 32);
    G1Affine pi;
    open_dev(&ctx->c, srs->s, dc, n, zz, &v, &pi, s);
    std::memcpy(value, &v, 32);
    store_proj(pi, proof);
    return TNS_OK;
  });
}

int tns_commitment_hash(const uint64_t proj[12], uint64_t out[4]) {
  return guarded([&]() {
    Fr h = commitment_hash(proj_to_affine_host(proj));
    std::memcpy(out, &h, 32);
    return TNS_OK;
  });
}

int tns_interpolate_consecutive(tns_ctx *ctx, const uint64_t *y, size_t n, uint64_t *coeffs) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    if (n == 0) return TNS_OK;
    DevBuf dy, dc;
    Fr *py = (Fr *)dy.ensure(sizeof(Fr) * n), *pc = (Fr *)dc.ensure(sizeof(Fr) * n);
    TNS_HIP(hipMemcpyAsync(py, y, sizeof(Fr) * n, hipMemcpyHostToDevice, ctx->c.stream));
    interpolate_consecutive_dev(&ctx->c, py, n, pc);
    TNS_HIP(hipMemcpyAsync(coeffs, pc, sizeof(Fr) * n, hipMemcpyDeviceToHost, ctx->c.stream));
    TNS_HIP(hipStreamSynchronize(ctx->c.stream));
    return TNS_OK;
  });
}

// The 2^nv-entry table of an MLE from the caller's n_evals entries: entries past n_evals are
// zero (the reference's evaluate sums over the entries it holds, src/polynomials.rs:91-102);
// more than 2^nv entries is rejected (callers fold aliases first).
static Fr *upload_mle(tns_ctx *ctx, const uint64_t *evals, size_t n_evals, unsigned nv, DevBuf &d) {
  if (nv > 30) throw Error(TNS_ERR_INVALID_PARAMETERS, "too many variables");
  const size_t n = (size_t)1 << nv;
  if (n_evals > n) throw Error(TNS_ERR_INVALID_PARAMETERS, "more evaluations than 2^num_vars");
  Fr *pe = (Fr *)d.ensure(sizeof(Fr) * n);
  if (n_evals) TNS_HIP(hipMemcpyAsync(pe, evals, sizeof(Fr) * n_evals, hipMemcpyHostToDevice, ctx->c.stream));
  if (n_evals < n) TNS_HIP(hipMemsetAsync(pe + n_evals, 0, sizeof(Fr) * (n - n_evals), ctx->c.stream));
  return pe;
}

int tns_mle_evaluate(tns_ctx *ctx, const uint64_t *evals, size_t n_evals, unsigned nv, const uint64_t *point,
                     uint64_t out[4]) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    DevBuf d;
    Fr *pe = upload_mle(ctx, evals, n_evals, nv, d);
    std::vector<Fr> pt(nv ? nv : 1);
    if (nv) std::memcpy(pt.data(), point, 32 * (size_t)nv);
    Fr r = mle_evaluate_dev(&ctx->c, pe, nv, pt.data());
    std::memcpy(out, &r, 32);
    return TNS_OK;
  });
}

int tns_mle_partial_evaluate(tns_ctx *ctx, const uint64_t *evals, size_t n_evals, unsigned nv,
                             const uint64_t *fixed, unsigned k, uint64_t *out) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    if (k > nv) throw Error(TNS_ERR_INVALID_PARAMETERS, "Cannot fix more variables than available");
    const size_t n = (size_t)1 << nv;
    DevBuf a, b;
    Fr *pa = upload_mle(ctx, evals, n_evals, nv, a);
    Fr *pb = (Fr *)b.ensure(sizeof(Fr) * (n / 2 + 1));
    Fr *src = pa, *dst = pb;
    for (unsigned j = 0; j < k; j++) {
      Fr r;
      std::memcpy(&r, fixed + 4 * (size_t)j, 32);
      mle_fold_dev(&ctx->c, src, dst, n >> (j + 1), r);
      std::swap(src, dst);
    }
    TNS_HIP(hipMemcpyAsync(out, src, sizeof(Fr) * (n >> k), hipMemcpyDeviceToHost, ctx->c.stream));
    TNS_HIP(hipStreamSynchronize(ctx->c.stream));
    return TNS_OK;
  });
}

tns_transcript *tns_transcript_new(const uint8_t seed[32]) {
  (void)seed;  // src/utils.rs:141-147: the seeded rng is replaced before first use
  return new tns_transcript();
}
void tns_transcript_free(tns_transcript *t) { delete t; }
void tns_transcript_append_field_element(tns_transcript *t, const uint8_t *label, size_t len, const uint64_t x[4]) {
  t->t.append_bytes(label, len);
  Fr f;
  std::memcpy(&f, x, 32);
  t->t.append_fr(f);
}
void tns_transcript_append_field_elements(tns_transcript *t, const uint8_t *label, size_t len,
                                          const uint64_t *xs, size_t n) {
  t->t.append_bytes(label, len);
  for (size_t i = 0; i < n; i++) {
    Fr f;
    std::memcpy(&f, xs + 4 * i, 32);
    t->t.append_fr(f);
  }
}
void tns_transcript_challenge_field_element(tns_transcript *t, const uint8_t *label, size_t len, uint64_t out[4]) {
  Fr r = t->t.challenge_bytes(label, len);
  std::memcpy(out, &r, 32);
}

static int sumcheck_prove_core(tns_ctx *ctx, Fr *const *ptrs, int n_tables, unsigned nv, const uint64_t claimed[4],
                               const tns_term *terms, int n_terms, tns_transcript *tr, uint64_t *rounds_out,
                               uint64_t final_out[4], uint64_t *challenges_out) {
  std::vector<SumcheckTerm> st(n_terms);
  for (int t = 0; t < n_terms; t++) {
    std::memcpy(&st[t].coeff, terms[t].coeff, 32);
    for (int j = 0; j < 3; j++) st[t].tab[j] = terms[t].tables[j];
  }
  Fr cl;
  std::memcpy(&cl, claimed, 32);
  std::vector<Fr> rounds(4 * (size_t)(nv ? nv : 1)), chal(nv ? nv : 1);
  Fr finals[4], fe;
  int rc = sumcheck_prove_dev(&ctx->c, ptrs, n_tables, nv, cl, st.data(), n_terms, tr->t, rounds.data(),
                              chal.data(), finals, &fe);
  std::memcpy(rounds_out, rounds.data(), 128 * (size_t)nv);
  if (challenges_out) std::memcpy(challenges_out, chal.data(), 32 * (size_t)nv);
  std::memcpy(final_out, &fe, 32);
  return rc;
}

static void check_sumcheck_shape(unsigned nv, int n_tables, int n_terms) {
  if (nv > 30 || n_tables < 0 || n_tables > 4 || n_terms < 0)
    throw Error(TNS_ERR_INVALID_PARAMETERS, "unsupported sum-check shape (<= 4 tables)");
}

int tns_sumcheck_prove(tns_ctx *ctx, const uint64_t *const *tables, int n_tables, unsigned nv,
                       const uint64_t claimed[4], const tns_term *terms, int n_terms, tns_transcript *tr,
                       uint64_t *rounds_out, uint64_t final_out[4], uint64_t *challenges_out) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    check_sumcheck_shape(nv, n_tables, n_terms);
    size_t n = (size_t)1 << nv;
    std::vector<DevBuf> bufs(n_tables);
    std::vector<Fr *> ptrs(n_tables);
    for (int i = 0; i < n_tables; i++) {
      ptrs[i] = (Fr *)bufs[i].ensure(sizeof(Fr) * n);
      TNS_HIP(hipMemcpyAsync(ptrs[i], tables[i], sizeof(Fr) * n, hipMemcpyHostToDevice, ctx->c.stream));
    }
    return sumcheck_prove_core(ctx, ptrs.data(), n_tables, nv, claimed, terms, n_terms, tr, rounds_out, final_out,
                               challenges_out);
  });
}

int tns_composition_sum_device(tns_ctx *ctx, const uint64_t *const *d_tables, int n_tables, unsigned nv,
                               const tns_term *terms, int n_terms, uint64_t out[4]) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    check_sumcheck_shape(nv, n_tables, n_terms);
    std::vector<Fr *> ptrs(n_tables);
    for (int i = 0; i < n_tables; i++) ptrs[i] = (Fr *)d_tables[i];
    std::vector<SumcheckTerm> st(n_terms);
    for (int t = 0; t < n_terms; t++) {
      std::memcpy(&st[t].coeff, terms[t].coeff, 32);
      for (int j = 0; j < 3; j++) st[t].tab[j] = terms[t].tables[j];
    }
    const Fr s = composition_sum_dev(&ctx->c, ptrs.data(), n_tables, nv, st.data(), n_terms);
    std::memcpy(out, &s, 32);
    return TNS_OK;
  });
}

int tns_sumcheck_prove_device(tns_ctx *ctx, const uint64_t *const *d_tables, int n_tables, unsigned nv,
                              const uint64_t claimed[4], const tns_term *terms, int n_terms, tns_transcript *tr,
                              uint64_t *rounds_out, uint64_t final_out[4], uint64_t *challenges_out) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    check_sumcheck_shape(nv, n_tables, n_terms);
    std::vector<Fr *> ptrs(n_tables);
    for (int i = 0; i < n_tables; i++) ptrs[i] = (Fr *)d_tables[i];  // only read
    return sumcheck_prove_core(ctx, ptrs.data(), n_tables, nv, claimed, terms, n_terms, tr, rounds_out, final_out,
                               challenges_out);
  });
}

int tns_last_prove_timing(tns_ctx *ctx, double out_ms[6]) {
  for (int i = 0; i < 6; i++) out_ms[i] = ctx->timing[i];
  return TNS_OK;
}

// ---------------------------------------------------------------- protocols
// Sum-check over the (zero) constraint closure + the two openings, for the rank's slices.
// The first nv - log2(size) rounds bind variables inside every slice (LSB-first,
// src/polynomials.rs:111-119), so they run locally; the last log2(size) rounds run on
// the host over the one folded value per table and rank (allgathered).
// flags (optional): the last of the mles as 0/1 bytes (sumcheck_zero_folds_async)
static void fill_common_tail(Ctx *c, const Srs &srs, HostTranscript &tr, Fr *const *mles, int n_mles,
                             unsigned nv, EvalPoly &polyA, EvalPoly &polyB, tns_proof *out, double *timing,
                             DevBuf &sbuf, Comm &m, const uint8_t *flags = nullptr, size_t n_flags = 0) {
  Timer t_sc;
  unsigned lr = 0;
  while ((1 << lr) < m.size) lr++;
  const unsigned nv_loc = nv - lr;  // check_shard guarantees size <= 2^nv
  if (n_mles < 1 || n_mles > 3) throw Error(TNS_ERR_INVALID_PARAMETERS, "1 to 3 trace tables");
  // The zero constraint closure (src/twist.rs:186-214, src/shout.rs:160-184) makes every round
  // polynomial [0, 0, 0, 0] and final_evaluation 0 (src/sumcheck.rs:77-104), so the transcript
  // alone yields the challenges: all nv rounds run on the host first ...
  const unsigned nv1 = nv ? nv : 1;
  std::vector<Fr> rounds(4 * (size_t)nv1, Fr::zero());
  Fr *chal = (Fr *)c->sc_host.ensure(sizeof(Fr) * (nv1 + 4)), *vals = chal + nv1;
  char lab[64];
  for (unsigned rnd = 0; rnd < nv; rnd++) {
    snprintf(lab, sizeof lab, "sumcheck_round_%u", rnd);  // src/sumcheck.rs:90-96
    tr.append_label(lab);
    for (int x = 0; x < 4; x++) tr.append_fr(Fr::zero());
    snprintf(lab, sizeof lab, "sumcheck_challenge_%u", rnd);
    chal[rnd] = tr.challenge(lab);
  }
  // ... and the folds binding this rank's tables at r_0 .. r_{nv_loc-1} (the MLE values the
  // closure evaluates, src/sumcheck.rs:104) run on the side stream under the openings; their
  // values are collected at the end of the proof
  // (queued behind the quotient kernel instead, under the opening sorts: a tie, 49.19-49.51 vs
  // 49.32-49.51 ms per step, profiles/r04_ab_folds_at.txt)
  // (queued once the openings' barycentric pass is on the device: its launches come first, and the
  // folds' ~80 us of host launches run under its chain kernels, profiles/r06_hiptrace_gaps.txt)
  Fr *d_vals = (Fr *)c->sc_out.ensure(sizeof(Fr) * 4);
  {
    hipEvent_t ready;
    TNS_HIP(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
    TNS_HIP(hipEventRecord(ready, c->stream));  // the tables were written on the context stream
    TNS_HIP(hipStreamWaitEvent(c->side, ready, 0));
    (void)hipEventDestroy(ready);
  }
  bool folds_queued = false;
  auto queue_folds = [&]() {
    if (folds_queued) return;
    folds_queued = true;
    sumcheck_zero_folds_async(c, c->side, mles, n_mles, nv_loc, chal, d_vals, flags, n_flags);
    TNS_HIP(hipMemcpyAsync(vals, d_vals, sizeof(Fr) * n_mles, hipMemcpyDeviceToHost, c->side));
  };
  const Fr fe = Fr::zero();
  out->num_rounds = nv;
  std::memcpy(out->round_polynomials, rounds.data(), 128 * (size_t)nv);
  std::memcpy(out->sumcheck_challenges, chal, 32 * (size_t)nv);
  std::memcpy(out->final_evaluation, &fe, 32);
  timing[3] = t_sc.ms();
  // challenge_field_elements("opening_challenges", nv) (src/utils.rs:195-203); only [0] is used
  // (src/twist.rs:219-226, src/shout.rs:189-195), and elements 1..nv-1 only extend a transcript
  // that nothing reads afterwards, so they are not derived (no observable output depends on
  // them; ~0.1 ms of host hashing in front of the openings at nv = 24)
  Timer t_open;
  // sharded: every rank's folded values travel with the opening partials (one exchange, not two)
  Fr finals[3];
  ExtraPayload fold_x;
  fold_x.data = finals;
  fold_x.bytes = sizeof(Fr) * (size_t)n_mles;
  bool folds_exchanged = false;
  auto folds_ready = [&]() {
    queue_folds();
    TNS_HIP(hipStreamSynchronize(c->side));
    for (int j = 0; j < n_mles; j++) finals[j] = vals[j];
  };
  if (nv >= 1) {
    Fr z = tr.challenge("opening_challenges_0");
    std::memcpy(out->opening_point, &z, 32);
    Fr v[2];
    G1Affine pi[2];
    open_evals_pair(c, srs, polyA, polyB, z, v, pi, sbuf, c->prove_ws[10], m, lr ? &fold_x : nullptr, folds_ready,
                    queue_folds);
    folds_exchanged = lr > 0;
    store_proj(pi[0], out->opening_proofs[0]);
    store_proj(pi[1], out->opening_proofs[1]);
    std::memcpy(out->final_evaluations[0], &v[0], 32);
    std::memcpy(out->final_evaluations[1], &v[1], 32);
    out->num_openings = 2;
  }
  timing[4] = t_open.ms();
  // the side stream's bound table values; with several ranks each holds its slice's values at
  // r_0 .. r_{nv_loc-1}, and the last lr challenges fold the allgathered rank values
  folds_ready();
  if (lr) {
    std::vector<Fr> all((size_t)n_mles * m.size);  // rank-major
    if (folds_exchanged) std::memcpy(all.data(), fold_x.all.data(), sizeof(Fr) * all.size());
    else all = allgather_fr(c, m, finals, (size_t)n_mles, "sum-check folded table values");
    for (int j = 0; j < n_mles; j++) {
      std::vector<Fr> t(m.size);
      for (int r = 0; r < m.size; r++) t[r] = all[(size_t)r * n_mles + j];
      for (unsigned rnd = nv_loc; rnd < nv; rnd++) {  // T'[s] = T[2s] + r (T[2s+1] - T[2s])
        const size_t h = t.size() / 2;
        for (size_t q = 0; q < h; q++) t[q] = add(t[2 * q], mul(chal[rnd], sub(t[2 * q + 1], t[2 * q])));
        t.resize(h);
      }
      finals[j] = t[0];
    }
  }
  for (int j = 0; j < n_mles; j++) std::memcpy(out->final_mle_evals[j], &finals[j], 32);
}

__global__ void k_write_flags(const uint8_t *__restrict__ in, Fr *__restrict__ out, size_t n_in, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = (i < n_in && in[i]) ? Fr::one() : Fr::zero();
}

__global__ void k_max_index_check(const uint64_t *__restrict__ idx, size_t n, uint64_t bound,
                                  unsigned *__restrict__ bad) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    if (idx[i] >= bound) *bad = 1;
}

// On every exit of a prove call (an exception included): nothing this call queued on the side
// stream (the flag table, the zero-closure folds: they read the caller's value / is_write
// buffers in the device-resident entry points) is still running when the call returns.
// The node ranges the drop-in values arrive in: k equal ranges (Ctx::upload_chunks).  (Splitting the
// last one in two, so the MSM left after the upload is an eighth of the vector, measured equal at
// C4: 56.4-57.5 vs 56.4-57.9 ms per drop-in proof, profiles/r04_ab_upload_split.txt.)
static std::vector<size_t> upload_chunk_offsets(size_t n, int k) {
  std::vector<size_t> off;
  const size_t per = (n + k - 1) / std::max(k, 1);
  for (size_t o = 0; o < n; o += per) off.push_back(o);
  off.push_back(n);
  return off;
}

struct SideDrain {
  Ctx *c;
  ~SideDrain() { (void)hipStreamSynchronize(c->side); }
};

// Twist::prove (src/twist.rs:107-252) for this rank's slice of the trace: operations
// [rank L, rank L + n_local) of n_total, L = next_pow2(n_total) / size.  kind: where
// addr/value/is_write live (H2D or D2D).  size 1 = the unsharded prover.
static void twist_core(tns_ctx *ctx, const tns_srs *srs, const tns_params *params, Comm &m, const uint64_t *addr,
                       const uint64_t *value, const uint8_t *is_write, size_t n_ops, uint64_t n_total,
                       tns_proof *out, hipMemcpyKind kind) {
  Timer total;
  CtxScope g(&ctx->c);
  Ctx *c = &ctx->c;
  hipStream_t st = c->stream;
  std::memset(out, 0, sizeof *out);
  if (n_total > params->max_operations)  // src/twist.rs:108-112
    throw Error(TNS_ERR_INVALID_PARAMETERS, "Too many operations");
  const size_t N = next_pow2(n_total);  // :141 next_power_of_two().max(1)
  const unsigned nv = ilog2_exact(N);
  if (nv > TNS_MAX_ROUNDS) throw Error(TNS_ERR_INVALID_PARAMETERS, "trace too long");
  check_shard(m, N, "trace");
  const size_t L = N / m.size, first = (size_t)m.rank * L;
  if (n_ops != slice_count(n_total, first, L))
    throw Error(TNS_ERR_INVALID_PARAMETERS, "local operation count does not match this rank's slice");
  double *tm = ctx->timing;
  for (int i = 0; i < 6; i++) tm[i] = 0;
  TNS_HIP(hipStreamSynchronize(c->side));  // a failed earlier proof's folds may still read the tables
  SideDrain drain{c};
  HostUpload upload(c);  // host inputs: addresses, flags, then values (under the address commitment)
  // ---- SoA extraction / padding into the resident workspace (src/twist.rs:115-148)
  Timer t_h2d;
  DevBuf &d_addr_raw = c->prove_ws[0], &d_flags = c->prove_ws[1], &d_a = c->prove_ws[2],
         &d_v = c->prove_ws[3], &d_o = c->prove_ws[4], &d_ca = c->prove_ws[5], &d_cv = c->prove_ws[6],
         &d_s = c->prove_ws[7];
  // V: a resident full slice is used in place (nothing below writes it); host input or a
  // padded slice goes through the workspace
  const bool v_in_place = kind == hipMemcpyDeviceToDevice && n_ops == L;
  Fr *A = (Fr *)d_a.ensure(sizeof(Fr) * L), *O = nullptr;
  Fr *V = v_in_place ? (Fr *)const_cast<uint64_t *>(value) : (Fr *)d_v.ensure(sizeof(Fr) * L);
  const uint64_t *ar = addr;
  const uint8_t *fl = is_write;
  // host inputs go through HostUpload (upload.cpp) on the copy stream, in the order the proof
  // needs them: the addresses (the first commitment starts on them), the flags, then the values
  // (32 B an op, 4x the addresses), whose copy runs under the address commitment -- the value MSM
  // is `late` in commit_evals_pair and waits for it
  const bool v_late = kind == hipMemcpyHostToDevice && n_ops > 0;
  int up_a = -1, up_f = -1, up_v = -1;
  // the values arrive in v_chunks node ranges, each committed as it lands (tns_ctx_set_upload_chunks,
  // default 4; 1 = one upload, one MSM after it); padded slices (L > n_ops) keep one MSM
  const std::vector<size_t> v_off =
      upload_chunk_offsets(n_ops, v_late && L == n_ops && n_ops >= ((size_t)1 << 18) ? c->upload_chunks : 1);
  const int v_chunks = std::max(1, (int)v_off.size() - 1);  // ranges actually formed
  uint32_t *dar32 = nullptr;
  // the op-type table is read by the sum-check only: its first fold pass reads the flag bytes
  // themselves (sumcheck_folds_take_flag_bytes), else it is written on the side stream
  unsigned lr = 0;
  while ((1 << lr) < m.size) lr++;
  const bool flag_bytes = sumcheck_folds_take_flag_bytes(nv - lr);
  if (kind == hipMemcpyHostToDevice) {
    uint64_t *dar = (uint64_t *)d_addr_raw.ensure(8 * (n_ops ? n_ops : 1));
    uint8_t *dfl = (uint8_t *)d_flags.ensure(n_ops ? n_ops : 1);
    if (n_ops) {
      // the addresses cross PCIe as u32 when they fit (memory sizes < 2^32: 64 MB fewer at 2^24 ops)
      dar32 = (uint32_t *)c->prove_ws[11].ensure(4 * n_ops);
      up_a = upload.add_narrow(dar32, dar, addr, n_ops);
      // flags read by the folds only (after both commitments) go last: their copy then runs under
      // the last value chunk's MSM instead of ahead of the values
      if (!flag_bytes) up_f = upload.add(dfl, is_write, n_ops);
      for (int k = 0; k < v_chunks; k++) {  // item ids up_v, up_v + 1, ...
        const int id = upload.add(V + v_off[k], value + 4 * v_off[k], sizeof(Fr) * (v_off[k + 1] - v_off[k]));
        if (k == 0) up_v = id;
      }
      if (flag_bytes) up_f = upload.add(dfl, is_write, n_ops);
      upload.start();
    }
    ar = dar;
    fl = dfl;
  } else if (n_ops && !v_in_place) {
    TNS_HIP(hipMemcpyAsync(V, value, sizeof(Fr) * n_ops, kind, st));
  }
  if (L > n_ops) fr_fill_zero_dev(c, V + n_ops, L - n_ops);
  if (!flag_bytes) {
    O = (Fr *)d_o.ensure(sizeof(Fr) * L);
    if (up_f >= 0) upload.wait(up_f, st);
    hipEvent_t in_ready;
    TNS_HIP(hipEventCreateWithFlags(&in_ready, hipEventDisableTiming));
    TNS_HIP(hipEventRecord(in_ready, st));
    TNS_HIP(hipStreamWaitEvent(c->side, in_ready, 0));
    (void)hipEventDestroy(in_ready);
    k_write_flags<<<grid_for(L, 256), 256, 0, c->side>>>(fl, O, n_ops, L);
    TNS_LAUNCH_CHECK();
  }
  if (kind == hipMemcpyHostToDevice) TNS_HIP(hipStreamSynchronize(st));
  tm[0] = t_h2d.ms();
  // the address table (Montgomery, for the sum-check and the openings) and its bit length are
  // written on lane 0 as its MSM starts, so the value commitment's lane does not wait for them;
  // the commitment's sort reads the raw u64 addresses (8 bytes a scalar, no canonical copy)
  unsigned *a_bits = (unsigned *)c->prove_ws[9].ensure(sizeof(unsigned));
  ScalarSource src_a;
  src_a.prep = [=, &upload](hipStream_t s) {
    if (up_a >= 0) {
      upload.wait(up_a, s);
      widen_dev(s, dar32, upload.narrow_width(up_a), n_ops, const_cast<uint64_t *>(ar));
    }
    u64_tables_dev(s, ar, n_ops, L, A, nullptr, a_bits);
  };
  src_a.canon_bits = a_bits;
  src_a.u64 = ar;
  src_a.n_u64 = n_ops;
  // ---- vector_to_polynomial + commit x2 (src/twist.rs:151-163).  The sum-check below
  // reads A and V without overwriting them, so the openings use the same vectors.
  Timer t_int;
  EvalPoly pa, pv;
  pa.N = pv.N = N;
  pa.first = pv.first = first;
  pa.cnt = pv.cnt = L;
  pa.coeffs = m.size == 1 ? (Fr *)d_ca.ensure(sizeof(Fr) * N) : nullptr;
  pv.coeffs = m.size == 1 ? (Fr *)d_cv.ensure(sizeof(Fr) * N) : nullptr;
  pa.y = A;
  pv.y = V;
  tm[1] = t_int.ms();
  Timer t_com;
  G1Affine cm[2];
  ScalarSource src_v;
  if (v_late) {
    src_v.prep = [&upload, up_v, v_chunks](hipStream_t s) {
      for (int k = 0; k < v_chunks; k++) upload.wait(up_v + k, s);
    };
    src_v.late = true;
    if (v_chunks > 1 && m.size == 1) {
      src_v.chunks = v_chunks;
      src_v.chunk_off = v_off;
      src_v.chunk_prep = [&upload, up_v](int k, hipStream_t s) { upload.wait(up_v + k, s); };
    }
  }
  commit_evals_pair(c, srs->s, pa, pv, m, cm, &src_a, v_late ? &src_v : nullptr);
  if (up_v >= 0) upload.wait_all(st);  // everything below on st / side reads the uploaded inputs
  const G1Affine Ca = cm[0], Cv = cm[1];
  store_proj(Ca, out->commitments[0]);
  store_proj(Cv, out->commitments[1]);
  tm[2] = t_com.ms();
  // ---- transcript (src/twist.rs:170-174)
  HostTranscript tr;
  tr.append_label("address_commitment");
  tr.append_fr(commitment_hash(Ca));
  tr.append_label("value_commitment");
  tr.append_fr(commitment_hash(Cv));
  // ---- sum-check over the addr / value / op-type MLEs + openings (src/twist.rs:177-243)
  Fr *mles[3] = {A, V, O};
  fill_common_tail(c, srs->s, tr, mles, 3, nv, pa, pv, out, tm, d_s, m, flag_bytes ? fl : nullptr, n_ops);
  TNS_HIP(hipStreamSynchronize(st));
  tm[5] = total.ms();
}

int tns_twist_prove(tns_ctx *ctx, const tns_srs *srs, const tns_params *params, const uint64_t *addr,
                    const uint64_t *value, const uint8_t *is_write, size_t n_ops, tns_proof *out) {
  return guarded([&]() {
    twist_core(ctx, srs, params, comm_self(), addr, value, is_write, n_ops, n_ops, out, hipMemcpyHostToDevice);
    return TNS_OK;
  });
}

int tns_twist_prove_device(tns_ctx *ctx, const tns_srs *srs, const tns_params *params, const uint64_t *d_addr,
                           const uint64_t *d_value, const uint8_t *d_is_write, size_t n_ops, tns_proof *out) {
  return guarded([&]() {
    twist_core(ctx, srs, params, comm_self(), d_addr, d_value, d_is_write, n_ops, n_ops, out,
               hipMemcpyDeviceToDevice);
    return TNS_OK;
  });
}

int tns_twist_prove_sharded(tns_ctx *ctx, const tns_srs *srs, const tns_params *params, tns_comm *comm,
                            const uint64_t *d_addr, const uint64_t *d_value, const uint8_t *d_is_write,
                            size_t n_local, uint64_t n_total, tns_proof *out) {
  return guarded([&]() {
    if (!comm || !comm->c) throw Error(TNS_ERR_INVALID_PARAMETERS, "null communicator");
    twist_core(ctx, srs, params, *comm->c, d_addr, d_value, d_is_write, n_local, n_total, out,
               hipMemcpyDeviceToDevice);
    return TNS_OK;
  });
}

// Shout::prove (src/shout.rs:97-222) for this rank's slices of the table (T) and the lookup
// index vector (M), sliced like twist_core's trace.
static void shout_core(tns_ctx *ctx, const tns_srs *srs, const tns_params *params, Comm &m, const uint64_t *entries,
                       size_t n_entries, uint64_t n_entries_total, const uint64_t *indices, size_t n_lookups,
                       uint64_t n_lookups_total, tns_proof *out, hipMemcpyKind kind) {
  Timer total;
  CtxScope g(&ctx->c);
  Ctx *c = &ctx->c;
  hipStream_t st = c->stream;
  std::memset(out, 0, sizeof *out);
  if (n_lookups_total > params->max_operations)  // src/shout.rs:98-102
    throw Error(TNS_ERR_INVALID_PARAMETERS, "Too many lookup operations");
  const size_t T = next_pow2(n_entries_total), M = next_pow2(n_lookups_total);  // :105, :116
  const unsigned nv = ilog2_exact(M);
  if (nv > TNS_MAX_ROUNDS) throw Error(TNS_ERR_INVALID_PARAMETERS, "too many lookups");
  check_shard(m, T, "table");
  check_shard(m, M, "lookup");
  const size_t LT = T / m.size, LM = M / m.size, firstT = (size_t)m.rank * LT, firstM = (size_t)m.rank * LM;
  if (n_entries != slice_count(n_entries_total, firstT, LT) || n_lookups != slice_count(n_lookups_total, firstM, LM))
    throw Error(TNS_ERR_INVALID_PARAMETERS, "local table / lookup count does not match this rank's slice");
  double *tm = ctx->timing;
  for (int i = 0; i < 6; i++) tm[i] = 0;
  TNS_HIP(hipStreamSynchronize(c->side));  // a failed earlier proof's folds may still read the tables
  SideDrain drain{c};
  HostUpload upload(c);  // host inputs: lookup indices, then the table (under the index commitment)
  Timer t_h2d;
  DevBuf &d_idx_raw = c->prove_ws[0], &d_bad = c->prove_ws[1], &d_t = c->prove_ws[2], &d_i = c->prove_ws[3],
         &d_ct = c->prove_ws[5], &d_ci = c->prove_ws[6], &d_s = c->prove_ws[7];
  Fr *TB = (Fr *)d_t.ensure(sizeof(Fr) * LT), *I = (Fr *)d_i.ensure(sizeof(Fr) * LM);
  if (LT > n_entries) fr_fill_zero_dev(c, TB + n_entries, LT - n_entries);  // the padding (src/shout.rs:105-107)
  const bool t_late = kind == hipMemcpyHostToDevice && n_entries > 0;
  int up_i = -1, up_t = -1;
  const uint64_t *ir = indices;
  uint32_t *dir32 = nullptr;
  if (kind == hipMemcpyHostToDevice) {
    if (n_lookups) {
      uint64_t *dir = (uint64_t *)d_idx_raw.ensure(8 * n_lookups);
      dir32 = (uint32_t *)c->prove_ws[11].ensure(4 * n_lookups);  // u32 over PCIe when they fit
      up_i = upload.add_narrow(dir32, dir, indices, n_lookups);
      ir = dir;
    }
    if (t_late) up_t = upload.add(TB, entries, sizeof(Fr) * n_entries);
    upload.start();
  } else if (n_entries) {
    TNS_HIP(hipMemcpyAsync(TB, entries, sizeof(Fr) * n_entries, kind, st));
  }
  // LookupTable::lookup bounds (src/shout.rs:44-50), agreed over the ranks
  unsigned hbad = 0;
  if (n_lookups) {
    if (up_i >= 0) {
      upload.wait(up_i, st);
      widen_dev(st, dir32, upload.narrow_width(up_i), n_lookups, const_cast<uint64_t *>(ir));
    }
    unsigned *bad = (unsigned *)d_bad.ensure(sizeof(unsigned));
    TNS_HIP(hipMemsetAsync(bad, 0, sizeof(unsigned), st));
    k_max_index_check<<<grid_for(n_lookups, 256), 256, 0, st>>>(ir, n_lookups, n_entries_total, bad);
    TNS_LAUNCH_CHECK();
    TNS_HIP(hipMemcpyAsync(&hbad, bad, sizeof hbad, hipMemcpyDeviceToHost, st));
    TNS_HIP(hipStreamSynchronize(st));
  }
  // (sharded: every rank's verdict travels with the commitments' partial sums and all ranks fail
  // together after that exchange -- the MSMs read the indices as scalars only, so an out-of-range
  // index is harmless until then, and a rank failing alone here would leave its peers waiting)
  if (hbad && m.size == 1) throw Error(TNS_ERR_INVALID_PARAMETERS, "Lookup index out of bounds");
  if (kind == hipMemcpyHostToDevice) TNS_HIP(hipStreamSynchronize(st));
  tm[0] = t_h2d.ms();
  // the index table is written on lane 1 as the index commitment starts (see twist_core)
  unsigned *i_bits = (unsigned *)c->prove_ws[9].ensure(sizeof(unsigned));
  ScalarSource src_i;
  src_i.prep = [=](hipStream_t s) { u64_tables_dev(s, ir, n_lookups, LM, I, nullptr, i_bits); };
  src_i.canon_bits = i_bits;
  src_i.u64 = ir;
  src_i.n_u64 = n_lookups;
  Timer t_int;
  EvalPoly pt, pi;
  pt.N = T;
  pi.N = M;
  pt.first = firstT;
  pi.first = firstM;
  pt.cnt = LT;
  pi.cnt = LM;
  pt.coeffs = m.size == 1 ? (Fr *)d_ct.ensure(sizeof(Fr) * T) : nullptr;
  pi.coeffs = m.size == 1 ? (Fr *)d_ci.ensure(sizeof(Fr) * M) : nullptr;
  pt.y = TB;
  pi.y = I;  // the sum-check leaves its input tables intact (mle.hip)
  tm[1] = t_int.ms();
  Timer t_com;
  G1Affine cm[2];
  ScalarSource src_t;
  if (t_late) {
    src_t.prep = [&upload, up_t](hipStream_t s) { upload.wait(up_t, s); };
    src_t.late = true;
  }
  ExtraPayload bad_x;
  bad_x.data = &hbad;
  bad_x.bytes = sizeof hbad;
  commit_evals_pair(c, srs->s, pt, pi, m, cm, t_late ? &src_t : nullptr, &src_i,
                    m.size > 1 ? &bad_x : nullptr);  // (src/shout.rs:125-133)
  if (up_t >= 0) upload.wait_all(st);
  if (m.size > 1) {  // LookupTable::lookup bounds (src/shout.rs:44-50), agreed over the ranks
    for (int r = 0; r < m.size; r++) {
      unsigned f;
      std::memcpy(&f, bad_x.all.data() + sizeof f * (size_t)r, sizeof f);
      hbad |= f;
    }
    if (hbad) throw Error(TNS_ERR_INVALID_PARAMETERS, "Lookup index out of bounds");
  }
  const G1Affine Ct = cm[0], Ci = cm[1];
  store_proj(Ct, out->commitments[0]);
  store_proj(Ci, out->commitments[1]);
  tm[2] = t_com.ms();
  HostTranscript tr;
  tr.append_label("table_commitment");
  tr.append_fr(commitment_hash(Ct));
  tr.append_label("index_commitment");
  tr.append_fr(commitment_hash(Ci));
  Fr *mles[1] = {I};  // the closure evaluates only the index MLE (src/shout.rs:175)
  fill_common_tail(c, srs->s, tr, mles, 1, nv, pt, pi, out, tm, d_s, m);
  TNS_HIP(hipStreamSynchronize(st));
  tm[5] = total.ms();
}

int tns_shout_prove(tns_ctx *ctx, const tns_srs *srs, const tns_params *params, const uint64_t *entries,
                    size_t n_entries, const uint64_t *indices, size_t n_lookups, tns_proof *out) {
  return guarded([&]() {
    shout_core(ctx, srs, params, comm_self(), entries, n_entries, n_entries, indices, n_lookups, n_lookups, out,
               hipMemcpyHostToDevice);
    return TNS_OK;
  });
}

int tns_shout_prove_device(tns_ctx *ctx, const tns_srs *srs, const tns_params *params, const uint64_t *d_entries,
                           size_t n_entries, const uint64_t *d_indices, size_t n_lookups, tns_proof *out) {
  return guarded([&]() {
    shout_core(ctx, srs, params, comm_self(), d_entries, n_entries, n_entries, d_indices, n_lookups, n_lookups,
               out, hipMemcpyDeviceToDevice);
    return TNS_OK;
  });
}

int tns_shout_prove_sharded(tns_ctx *ctx, const tns_srs *srs, const tns_params *params, tns_comm *comm,
                            const uint64_t *d_entries, size_t n_entries_local, uint64_t n_entries_total,
                            const uint64_t *d_indices, size_t n_lookups_local, uint64_t n_lookups_total,
                            tns_proof *out) {
  return guarded([&]() {
    if (!comm || !comm->c) throw Error(TNS_ERR_INVALID_PARAMETERS, "null communicator");
    shout_core(ctx, srs, params, *comm->c, d_entries, n_entries_local, n_entries_total, d_indices, n_lookups_local,
               n_lookups_total, out, hipMemcpyDeviceToDevice);
    return TNS_OK;
  });
}

// ---------------------------------------------------------------- verifiers (host)
static G2Affine g2_from_limbs(const uint64_t in[16]) {
  G2Affine g;
  std::memcpy(&g.x0, in, 32);
  std::memcpy(&g.x1, in + 4, 32);
  std::memcpy(&g.y0, in + 8, 32);
  std::memcpy(&g.y1, in + 12, 32);
  g.inf = g.x0.is_zero() && g.x1.is_zero() && g.y0.is_zero() && g.y1.is_zero();
  if (!g.inf && !g2_on_curve(g)) throw Error(TNS_ERR_INVALID_PARAMETERS, "G2 point not on the twist");
  return g;
}
static void g2_to_limbs(const G2Affine &g, uint64_t out[16]) {
  if (g.inf) {
    std::memset(out, 0, 128);
    return;
  }
  std::memcpy(out, &g.x0, 32);
  std::memcpy(out + 4, &g.x1, 32);
  std::memcpy(out + 8, &g.y0, 32);
  std::memcpy(out + 12, &g.y1, 32);
}
static G1Affine g1_from_limbs(const uint64_t in[8]) {
  G1Affine a;
  std::memcpy(&a.x, in, 32);
  std::memcpy(&a.y, in + 4, 32);
  if (!a.is_inf() && !g1_on_curve(a)) throw Error(TNS_ERR_INVALID_PARAMETERS, "G1 point not on the curve");
  return a;
}
struct Vk {
  G1Affine g1;
  G2Affine g2, g2_tau;
};
static Vk vk_load(const tns_vk *vk) { return Vk{g1_from_limbs(vk->g1), g2_from_limbs(vk->g2), g2_from_limbs(vk->g2_tau)}; }
static Fr fr_load(const uint64_t x[4]) {
  Fr r;
  std::memcpy(&r, x, 32);
  return r;
}

static int verify_proof(const tns_vk *vk, const tns_proof *p, const char *l0, const char *l1, int *ok) {
  return guarded([&]() {
    const Vk k = vk_load(vk);
    if (p->num_rounds > TNS_MAX_ROUNDS || p->num_openings > 2) throw Error(TNS_ERR_INVALID_PARAMETERS, "malformed proof");
    G1Affine C[2] = {proj_to_affine_host(p->commitments[0]), proj_to_affine_host(p->commitments[1])};
    G1Affine pi[2] = {proj_to_affine_host(p->opening_proofs[0]), proj_to_affine_host(p->opening_proofs[1])};
    Fr vals[2] = {fr_load(p->final_evaluations[0]), fr_load(p->final_evaluations[1])};
    std::vector<Fr> rounds(4 * (size_t)(p->num_rounds ? p->num_rounds : 1));
    std::memcpy(rounds.data(), p->round_polynomials, 128 * (size_t)p->num_rounds);
    *ok = protocol_verify_host(k.g1, k.g2, k.g2_tau, l0, l1, C, rounds.data(), p->num_rounds,
                               fr_load(p->final_evaluation), p->num_openings, pi, vals)
              ? 1 : 0;
    return TNS_OK;
  });
}

int tns_verifier_key(const tns_params *params, tns_vk *out) {
  return guarded([&]() {
    G1Affine g1;
    G2Affine g2, g2t;
    verifier_key(fr_load(params->tau), &g1, &g2, &g2t);
    std::memcpy(out->g1, &g1, 64);
    g2_to_limbs(g2, out->g2);
    g2_to_limbs(g2t, out->g2_tau);
    return TNS_OK;
  });
}

int tns_kzg_verify(const tns_vk *vk, const uint64_t commitment_proj[12], const uint64_t z[4], const uint64_t value[4],
                   const uint64_t proof_proj[12], int *ok) {
  return guarded([&]() {
    const Vk k = vk_load(vk);
    *ok = kzg_verify_host(k.g1, k.g2, k.g2_tau, proj_to_affine_host(commitment_proj), fr_load(z), fr_load(value),
                          proj_to_affine_host(proof_proj))
              ? 1 : 0;
    return TNS_OK;
  });
}

int tns_kzg_batch_verify(const tns_vk *vk, size_t n, const uint64_t *commitments_proj, const uint64_t *points,
                         const uint64_t *values, const uint64_t *proofs_proj, int *ok) {
  return guarded([&]() {
    const Vk k = vk_load(vk);
    std::vector<G1Affine> C(n), pi(n);
    std::vector<Fr> z(n), v(n);
    for (size_t i = 0; i < n; i++) {
      C[i] = proj_to_affine_host(commitments_proj + 12 * i);
      pi[i] = proj_to_affine_host(proofs_proj + 12 * i);
      z[i] = fr_load(points + 4 * i);
      v[i] = fr_load(values + 4 * i);
    }
    *ok = kzg_batch_verify_host(k.g1, k.g2, k.g2_tau, n, C.data(), z.data(), v.data(), pi.data()) ? 1 : 0;
    return TNS_OK;
  });
}

int tns_twist_verify(const tns_vk *vk, const tns_proof *proof, int *ok) {
  return verify_proof(vk, proof, "address_commitment", "value_commitment", ok);
}

int tns_shout_verify(const tns_vk *vk, const tns_proof *proof, int *ok) {
  return verify_proof(vk, proof, "table_commitment", "index_commitment", ok);
}

int tns_pairing(const uint64_t g1_affine[8], const uint64_t g2_affine[16], uint64_t out[48]) {
  return guarded([&]() {
    Fq e[12];
    pairing_value(g1_from_limbs(g1_affine), g2_from_limbs(g2_affine), e);
    std::memcpy(out, e, sizeof e);
    return TNS_OK;
  });
}

int tns_g2_mul(const uint64_t g2_affine[16], const uint64_t k[4], uint64_t out[16]) {
  return guarded([&]() {
    g2_to_limbs(g2_mul(g2_from_limbs(g2_affine), k), out);
    return TNS_OK;
  });
}

// ---------------------------------------------------------------- wire format (host)
int tns_g1_serialize(const uint64_t proj[12], int compressed, uint8_t *out) {
  return guarded([&]() {
    g1_serialize(proj_to_affine_host(proj), compressed != 0, out);
    return TNS_OK;
  });
}

int tns_g1_deserialize(const uint8_t *in, int compressed, uint64_t proj_out[12]) {
  return guarded([&]() {
    store_proj(g1_deserialize(in, compressed != 0, true), proj_out);
    return TNS_OK;
  });
}

namespace {
struct Writer {
  uint8_t *out;
  size_t cap, n = 0;
  void bytes(const uint8_t *p, size_t k) {
    if (out && n + k <= cap) std::memcpy(out + n, p, k);
    n += k;
  }
  void u64(uint64_t v) {
    uint8_t b[8];
    for (int i = 0; i < 8; i++) b[i] = (uint8_t)(v >> (8 * i));
    bytes(b, 8);
  }
};
struct Reader {
  const uint8_t *in;
  size_t len, n = 0;
  const uint8_t *take(size_t k) {
    if (n + k > len) throw Error(TNS_ERR_INVALID_PARAMETERS, "truncated proof bytes");
    const uint8_t *p = in + n;
    n += k;
    return p;
  }
  uint64_t u64() {
    const uint8_t *b = take(8);
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v |= (uint64_t)b[i] << (8 * i);
    return v;
  }
};
}  // namespace

int tns_proof_serialize(const tns_proof *p, int compressed, uint8_t *out, size_t cap, size_t *len) {
  return guarded([&]() {
    const size_t gs = compressed ? 32 : 64;
    Writer w{out, cap};
    uint8_t g[64], f[32];
    for (int i = 0; i < 2; i++) {
      g1_serialize(proj_to_affine_host(p->commitments[i]), compressed != 0, g);
      w.bytes(g, gs);
    }
    w.u64(p->num_rounds);
    for (uint32_t r = 0; r < p->num_rounds; r++) {
      w.u64(4);
      for (int x = 0; x < 4; x++) {
        fr_serialize(fr_load(p->round_polynomials[r][x]), f);
        w.bytes(f, 32);
      }
    }
    fr_serialize(fr_load(p->final_evaluation), f);
    w.bytes(f, 32);
    w.u64(p->num_openings);
    for (uint32_t i = 0; i < p->num_openings; i++) {
      g1_serialize(proj_to_affine_host(p->opening_proofs[i]), compressed != 0, g);
      w.bytes(g, gs);
    }
    w.u64(p->num_openings);  // final_evaluations has one value per opening
    for (uint32_t i = 0; i < p->num_openings; i++) {
      fr_serialize(fr_load(p->final_evaluations[i]), f);
      w.bytes(f, 32);
    }
    *len = w.n;
    if (out && w.n > cap) throw Error(TNS_ERR_INVALID_PARAMETERS, "output buffer too small");
    return TNS_OK;
  });
}

int tns_proof_deserialize(const uint8_t *in, size_t len, int compressed, tns_proof *p) {
  return guarded([&]() {
    std::memset(p, 0, sizeof *p);
    const size_t gs = compressed ? 32 : 64;
    Reader r{in, len};
    for (int i = 0; i < 2; i++) store_proj(g1_deserialize(r.take(gs), compressed != 0, true), p->commitments[i]);
    const uint64_t nr = r.u64();
    if (nr > TNS_MAX_ROUNDS) throw Error(TNS_ERR_INVALID_PARAMETERS, "too many sum-check rounds");
    p->num_rounds = (uint32_t)nr;
    for (uint64_t k = 0; k < nr; k++) {
      if (r.u64() != 4) throw Error(TNS_ERR_INVALID_PARAMETERS, "round polynomial must have 4 coefficients");
      for (int x = 0; x < 4; x++) {
        const Fr v = fr_deserialize(r.take(32));
        std::memcpy(p->round_polynomials[k][x], &v, 32);
      }
    }
    const Fr fe = fr_deserialize(r.take(32));
    std::memcpy(p->final_evaluation, &fe, 32);
    const uint64_t no = r.u64();
    if (no > 2) throw Error(TNS_ERR_INVALID_PARAMETERS, "more than two opening proofs");
    p->num_openings = (uint32_t)no;
    for (uint64_t i = 0; i < no; i++) store_proj(g1_deserialize(r.take(gs), compressed != 0, true), p->opening_proofs[i]);
    const uint64_t nf = r.u64();
    if (nf != no) throw Error(TNS_ERR_INVALID_PARAMETERS, "final evaluations do not match the openings");
    for (uint64_t i = 0; i < nf; i++) {
      const Fr v = fr_deserialize(r.take(32));
      std::memcpy(p->final_evaluations[i], &v, 32);
    }
    if (r.n != len) throw Error(TNS_ERR_INVALID_PARAMETERS, "trailing bytes after the proof");
    return TNS_OK;
  });
}

// ---------------------------------------------------------------- communicators
int tns_comm_unique_id(uint8_t uid[128]) {
  return guarded([&]() {
    comm_unique_id(uid);
    return TNS_OK;
  });
}

int tns_comm_create(tns_ctx *ctx, int rank, int size, const uint8_t uid[128], tns_comm **out) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    tns_comm *cm = new tns_comm();
    try {
      cm->c = comm_rccl_new(&ctx->c, rank, size, uid);
    } catch (...) {
      delete cm;
      throw;
    }
    *out = cm;
    return TNS_OK;
  });
}

int tns_comm_create_callback(int rank, int size, tns_allgather_fn fn, void *user, tns_comm **out) {
  return guarded([&]() {
    tns_comm *cm = new tns_comm();
    try {
      cm->c = comm_callback_new(rank, size, fn, user);
    } catch (...) {
      delete cm;
      throw;
    }
    *out = cm;
    return TNS_OK;
  });
}

void tns_comm_destroy(tns_comm *comm) { delete comm; }

int tns_comm_info(const tns_comm *comm, int *rank, int *size, int *seen_size, int *kind) {
  return guarded([&]() {
    if (!comm || !comm->c) throw Error(TNS_ERR_INVALID_PARAMETERS, "null communicator");
    if (rank) *rank = comm->c->rank;
    if (size) *size = comm->c->size;
    if (seen_size) *seen_size = comm->c->seen_size();
    if (kind) *kind = comm->c->kind();
    return TNS_OK;
  });
}

int tns_comm_allgather(tns_ctx *ctx, tns_comm *comm, const void *send, size_t bytes, void *recv) {
  return guarded([&]() {
    if (!comm || !comm->c) throw Error(TNS_ERR_INVALID_PARAMETERS, "null communicator");
    if (bytes && (!send || !recv)) throw Error(TNS_ERR_INVALID_PARAMETERS, "null exchange buffer");
    comm->c->exchange(ctx ? &ctx->c : nullptr, send, bytes, recv, "tns_comm_allgather");
    return TNS_OK;
  });
}

int tns_comm_set_timeout(tns_comm *comm, double seconds) {
  return guarded([&]() {
    if (!comm || !comm->c) throw Error(TNS_ERR_INVALID_PARAMETERS, "null communicator");
    if (!(seconds > 0.0)) throw Error(TNS_ERR_INVALID_PARAMETERS, "timeout must be positive");
    comm->c->timeout_s = seconds;
    return TNS_OK;
  });
}

int tns_comm_stats_ex(const tns_comm *comm, double out[6]) {
  return guarded([&]() {
    if (!comm || !comm->c || !out) throw Error(TNS_ERR_INVALID_PARAMETERS, "null communicator or output");
    out[0] = (double)comm->c->seq;
    out[1] = comm->c->total_s;
    out[2] = comm->c->max_s;
    out[3] = comm->c->timeout_s;
    out[4] = comm->c->bytes_total;
    out[5] = comm->c->bytes_max;
    return TNS_OK;
  });
}

int tns_comm_stats(const tns_comm *comm, double out[4]) {
  return guarded([&]() {
    if (!comm || !comm->c || !out) throw Error(TNS_ERR_INVALID_PARAMETERS, "null communicator or output");
    out[0] = (double)comm->c->seq;
    out[1] = comm->c->total_s;
    out[2] = comm->c->max_s;
    out[3] = comm->c->timeout_s;
    return TNS_OK;
  });
}

int tns_srs_prepare_lagrange_shard(tns_ctx *ctx, tns_srs *srs, size_t n, int rank, int size) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    if (!srs->s.has_tau) throw Error(TNS_ERR_INVALID_PARAMETERS, "SRS has no tau");
    if (n == 0 || (n & (n - 1))) throw Error(TNS_ERR_INVALID_PARAMETERS, "Lagrange basis size must be a power of two");
    if (size < 1 || (size & (size - 1)) || rank < 0 || rank >= size || (size_t)size > n)
      throw Error(TNS_ERR_INVALID_PARAMETERS, "bad shard");
    const bool saved = ctx->c.lagrange_commit;
    ctx->c.lagrange_commit = true;
    const size_t L = n / size;
    (void)lagrange_basis_dev(&ctx->c, srs->s, n, (size_t)rank * L, L);
    ctx->c.lagrange_commit = saved;
    return TNS_OK;
  });
}

// ---------------------------------------------------------------- device buffers
int tns_buffer_upload(tns_ctx *ctx, const void *host, size_t bytes, tns_buffer **out) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    tns_buffer *b = new tns_buffer();
    b->device = ctx->c.device;
    b->bytes = bytes;
    try {
      b->buf.ensure(bytes ? bytes : 16);
      if (bytes) TNS_HIP(hipMemcpy(b->buf.p, host, bytes, hipMemcpyHostToDevice));
    } catch (...) {
      delete b;
      throw;
    }
    *out = b;
    return TNS_OK;
  });
}
void *tns_buffer_device_ptr(const tns_buffer *b) { return b ? b->buf.p : nullptr; }
int tns_buffer_download(const tns_buffer *b, void *host, size_t bytes) {
  return guarded([&]() {
    if (!b || bytes > b->bytes) throw Error(TNS_ERR_INVALID_PARAMETERS, "download beyond the buffer");
    TNS_HIP(hipSetDevice(b->device));
    if (bytes) TNS_HIP(hipMemcpy(host, b->buf.p, bytes, hipMemcpyDeviceToHost));
    return TNS_OK;
  });
}
void tns_buffer_free(tns_buffer *b) {
  if (!b) return;
  (void)hipSetDevice(b->device);
  delete b;
}

int tns_msm_device(tns_ctx *ctx, const tns_srs *srs, const uint64_t *d_scalars, size_t n, uint64_t out[12]) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    store_proj(commit_dev(&ctx->c, srs->s, (const Fr *)d_scalars, n), out);
    return TNS_OK;
  });
}

int tns_msm_sharded(tns_ctx *ctx, const tns_srs *srs, tns_comm *comm, const uint64_t *d_scalars, size_t n_local,
                    uint64_t n_total, uint64_t out[12]) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    if (!comm || !comm->c) throw Error(TNS_ERR_INVALID_PARAMETERS, "null communicator");
    Comm &m = *comm->c;
    if (n_total > srs->s.n) throw Error(TNS_ERR_COMMITMENT, "Polynomial degree exceeds setup size");
    const size_t N = next_pow2((size_t)n_total);
    check_shard(m, N, "coefficient");
    const size_t L = N / (size_t)m.size, first = (size_t)m.rank * L;
    if (n_local != slice_count(n_total, first, L))
      throw Error(TNS_ERR_INVALID_PARAMETERS, "n_local is not this rank's slice of n_total");
    if (n_local && (first < srs->s.first || first + n_local > srs->s.first + srs->s.held))
      throw Error(TNS_ERR_INVALID_PARAMETERS, "this rank's SRS share does not hold its coefficient slice");
    const size_t off = first - std::min(first, srs->s.first);
    const FixedBase *fb = srs_fixed_base(&ctx->c, srs->s, n_local);
    const G1Xyzz part = n_local ? msm_dev(&ctx->c, srs->s.points.as<G1Affine>() + off, (const Fr *)d_scalars, n_local,
                                          fb, off)
                                : G1Xyzz::inf();
    store_proj(xyzz_to_affine(allgather_sum_g1(&ctx->c, m, part, "sharded MSM partial")), out);
    return TNS_OK;
  });
}

// ---------------------------------------------------------------- clock probe
// Every workgroup: a chain of `iters` Montgomery products per lane (the accumulation's
// instruction mix), bracketed by the shader-clock and constant 100 MHz counters.
__global__ void __launch_bounds__(256) k_clock_probe(uint32_t iters, uint32_t seed, uint64_t *__restrict__ out,
                                                     uint32_t *__restrict__ sink) {
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  Fq a, b;
#pragma unroll
  for (int l = 0; l < 8; l++) {
    a.v[l] = (seed + threadIdx.x * 0x9e3779b9u + l * 0x85ebca6bu) & (l == 7 ? 0x0fffffffu : 0xffffffffu);
    b.v[l] = (seed * 31u + blockIdx.x + l * 0xc2b2ae35u) & (l == 7 ? 0x0fffffffu : 0xffffffffu);
  }
  for (uint32_t i = 0; i < iters; i++) {
    a = mul(a, b);
    b = mul(b, a);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (a.v[0] == 0x12345678u && b.v[1] == 0x9abcdef0u) sink[0] = a.v[2];  // keep the chain live
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = t1 - t0;
    out[2 * blockIdx.x + 1] = r1 - r0;
  }
}

int tns_clock_probe(tns_ctx *ctx, double ms, double out[4]) {
  return guarded([&]() {
    if (!ctx || !out || !(ms > 0.0)) throw Error(TNS_ERR_INVALID_PARAMETERS, "null context/output or ms <= 0");
    CtxScope g(&ctx->c);
    hipStream_t st = ctx->c.stream;
    int cus = 0;
    TNS_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->c.device));
    const unsigned nblk = (unsigned)std::max(1, cus) * 4;  // 4 waves per SIMD
    DevBuf dout, dsink;
    uint64_t *d = (uint64_t *)dout.ensure(sizeof(uint64_t) * 2 * nblk);
    uint32_t *sink = (uint32_t *)dsink.ensure(sizeof(uint32_t));
    hipEvent_t e0, e1;
    TNS_HIP(hipEventCreate(&e0));
    TNS_HIP(hipEventCreate(&e1));
    auto run = [&](uint32_t iters) {
      TNS_HIP(hipEventRecord(e0, st));
      k_clock_probe<<<nblk, 256, 0, st>>>(iters, 0x1234567u, d, sink);
      TNS_LAUNCH_CHECK();
      TNS_HIP(hipEventRecord(e1, st));
      TNS_HIP(hipEventSynchronize(e1));
      float t = 0.f;
      TNS_HIP(hipEventElapsedTime(&t, e0, e1));
      return (double)t;
    };
    uint32_t iters = 256;
    double t = run(iters);
    while (t < ms / 4 && iters < (1u << 26)) {  // calibrate to about `ms`
      iters = (uint32_t)std::min<double>((double)(1u << 26), iters * std::max(2.0, 0.5 * ms / std::max(t, 1e-3)));
      t = run(iters);
    }
    if (t < ms) t = run((uint32_t)std::min<double>((double)(1u << 30), iters * ms / std::max(t, 1e-3)));
    std::vector<uint64_t> h(2 * nblk);
    TNS_HIP(hipMemcpy(h.data(), d, sizeof(uint64_t) * 2 * nblk, hipMemcpyDeviceToHost));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    std::vector<double> mhz;
    for (unsigned b = 0; b < nblk; b++)
      if (h[2 * b + 1]) mhz.push_back(100.0 * (double)h[2 * b] / (double)h[2 * b + 1]);
    if (mhz.empty()) throw Error(TNS_ERR_DEVICE, "clock probe: no workgroup reported");
    std::sort(mhz.begin(), mhz.end());
    out[0] = mhz[mhz.size() / 2];
    out[1] = mhz.front();
    out[2] = mhz.back();
    out[3] = t;
    return TNS_OK;
  });
}

// ---------------------------------------------------------------- kernel timing (HIP events)
int tns_profile_enable(tns_ctx *ctx, int on) {
  ctx->c.prof.enabled = on != 0;
  ctx->c.prof.only.clear();  // a new profile times every stage until tns_profile_only narrows it
  ctx->c.prof.start(ctx->c.stream);
  return TNS_OK;
}

int tns_profile_only(tns_ctx *ctx, const char *stage) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    ctx->c.prof.only = stage ? stage : "";
    return TNS_OK;
  });
}

int tns_profile_read_ex(tns_ctx *ctx, const char *stage, double out[5]) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    ctx->c.prof.collect();
    auto it = ctx->c.prof.totals.find(stage);
    const bool f = it != ctx->c.prof.totals.end();
    out[0] = f ? it->second.ms : 0.0;
    out[1] = f ? (double)it->second.launches : 0.0;
    out[2] = f ? it->second.bytes : 0.0;
    out[3] = f ? it->second.ops : 0.0;
    out[4] = f ? it->second.busy_ms : 0.0;
    return TNS_OK;
  });
}
int tns_profile_read(tns_ctx *ctx, const char *kernel, double *total_ms, uint64_t *launches, double *alg_bytes) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    ctx->c.prof.collect();
    auto it = ctx->c.prof.totals.find(kernel);
    bool f = it != ctx->c.prof.totals.end();
    *total_ms = f ? it->second.ms : 0.0;
    *launches = f ? it->second.launches : 0;
    *alg_bytes = f ? it->second.bytes : 0.0;
    return TNS_OK;
  });
}

// n draws of ark-ff UniformRand for Fr from one ChaCha20Rng::from_seed(seed) stream (host)
void tns_fr_rand_batch(const uint8_t seed[32], size_t n, uint64_t *out_mont) {
  host_fr_rand_stream(seed, n, (Fr *)out_mont);
}

// ---------------------------------------------------------------- host utilities
void tns_fr_from_u64(const uint64_t *in, size_t n, uint64_t *out) {
  par_convert<FrCfg>(in, n, out, [](const uint64_t *i, uint64_t *o, size_t k) {
    Fr r = from_u64<FrCfg>(i[k]);
    std::memcpy(o + 4 * k, &r, 32);
  });
}
void tns_fr_from_canonical(const uint64_t *in, size_t n, uint64_t *out) {
  par_convert<FrCfg>(in, n, out, [](const uint64_t *i, uint64_t *o, size_t k) {
    Fr x;
    std::memcpy(&x, i + 4 * k, 32);
    reduce_once(x);
    Fr r = to_mont(x);
    std::memcpy(o + 4 * k, &r, 32);
  });
}
void tns_fr_to_canonical(const uint64_t *in, size_t n, uint64_t *out) {
  par_convert<FrCfg>(in, n, out, [](const uint64_t *i, uint64_t *o, size_t k) {
    Fr x;
    std::memcpy(&x, i + 4 * k, 32);
    Fr r = from_mont(x);
    std::memcpy(o + 4 * k, &r, 32);
  });
}
void tns_fq_to_canonical(const uint64_t *in, size_t n, uint64_t *out) {
  par_convert<FqCfg>(in, n, out, [](const uint64_t *i, uint64_t *o, size_t k) {
    Fq x;
    std::memcpy(&x, i + 4 * k, 32);
    Fq r = from_mont(x);
    std::memcpy(o + 4 * k, &r, 32);
  });
}

// ProtocolBenchmarks trace (src/benchmarks.rs:88-99), operations [first, first + count) of
// an n_total-operation run (the memory state is replayed from operation 0)
static void bench_trace_core(size_t memory_size, uint64_t n_total, uint64_t first, size_t count, uint64_t *addr,
                             uint64_t *value, uint8_t *is_write) {
  if (memory_size == 0 || (memory_size & (memory_size - 1)))
    throw Error(TNS_ERR_INVALID_PARAMETERS, "Memory size must be power of 2");
  if (first + count > n_total) throw Error(TNS_ERR_INVALID_PARAMETERS, "slice beyond the trace");
  std::vector<uint64_t> mem(memory_size, 0);
  for (uint64_t i = 0; i < first + count; i++) {
    const bool out = i >= first;
    if (i % 3 == 0) {
      const size_t a = i % memory_size;
      mem[a] = i * 42;
      if (out) {
        addr[i - first] = a;
        value[i - first] = mem[a];
        is_write[i - first] = 1;
      }
    } else if (out) {
      const size_t a = (i / 2) % memory_size;
      addr[i - first] = a;
      value[i - first] = mem[a];
      is_write[i - first] = 0;
    }
  }
}

int tns_bench_trace(size_t memory_size, size_t n_ops, uint64_t *addr, uint64_t *value, uint8_t *is_write) {
  return guarded([&]() {
    bench_trace_core(memory_size, n_ops, 0, n_ops, addr, value, is_write);
    return TNS_OK;
  });
}

int tns_bench_trace_slice(size_t memory_size, uint64_t n_total, uint64_t first, size_t count, uint64_t *addr,
                          uint64_t *value, uint8_t *is_write) {
  return guarded([&]() {
    bench_trace_core(memory_size, n_total, first, count, addr, value, is_write);
    return TNS_OK;
  });
}

}  // extern "C"
