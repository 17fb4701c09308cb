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
// (vector_to_polynomial input, src/polynomials.rs:248-262).  Committed and opened via
// the Lagrange basis when the SRS provides it, else via interpolated coefficients.
struct EvalPoly {
  const Fr *y = nullptr;       // device, N (must stay intact until opened)
  Fr *coeffs = nullptr;        // device scratch, N (coefficient path)
  size_t N = 0;
  const LagrangeBasis *basis = nullptr;
  bool have_coeffs = false;
};

static G1Affine commit_evals(Ctx *c, const Srs &srs, EvalPoly &p) {
  if (p.N > srs.n) throw Error(TNS_ERR_COMMITMENT, "Polynomial degree exceeds setup size");
  p.basis = lagrange_basis_dev(c, srs, p.N);
  if (p.basis) return xyzz_to_affine(msm_dev(c, p.basis->points.as<G1Affine>(), p.y, p.N, p.basis->fb));
  interpolate_consecutive_dev(c, p.y, p.N, p.coeffs);
  p.have_coeffs = true;
  return commit_dev(c, srs, p.coeffs, p.N);
}

static void open_evals(Ctx *c, const Srs &srs, EvalPoly &p, const Fr &z, Fr *value, G1Affine *proof,
                       DevBuf &sbuf) {
  if (p.basis) {
    Fr *q = (Fr *)sbuf.ensure(sizeof(Fr) * p.N);
    if (lagrange_quotient_dev(c, p.y, p.N, z, value, q)) {
      *proof = xyzz_to_affine(msm_dev(c, p.basis->points.as<G1Affine>(), q, p.N, p.basis->fb));
      return;
    }
  }
  if (!p.have_coeffs) {  // z is a node (or no basis): coefficient form
    interpolate_consecutive_dev(c, p.y, p.N, p.coeffs);
    p.have_coeffs = true;
  }
  open_dev(c, srs, p.coeffs, p.N, z, value, proof, sbuf);
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

int tns_ctx_create(int device, tns_ctx **out) {
  return guarded([&]() {
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
    TNS_HIP(hipStreamCreateWithFlags(&x->c.stream, hipStreamNonBlocking));
    *out = x;
    return TNS_OK;
  });
}

void tns_ctx_destroy(tns_ctx *ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->c.device);
  (void)hipStreamSynchronize(ctx->c.stream);
  delete ctx;
}

int tns_ctx_synchronize(tns_ctx *ctx) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    TNS_HIP(hipStreamSynchronize(ctx->c.stream));
    return TNS_OK;
  });
}

int tns_setup_params(tns_ctx *ctx, unsigned log_size, tns_params *out, tns_srs **srs_out) {
  return guarded([&]() {
    if (log_size > 26) throw Error(TNS_ERR_INVALID_PARAMETERS, "log_size too large");
    std::memset(out, 0, sizeof *out);
    out->log_size = log_size;
    out->max_operations = (uint64_t)1 << (log_size + 2);  // src/utils.rs:80
    out->num_powers = next_pow2(out->max_operations) + 1;  // src/utils.rs:89
    uint8_t seed42[32];
    std::memset(seed42, 42, 32);
    Fr tau = host_fr_rand_chacha(seed42, out->fiat_shamir_seed);  // src/utils.rs:81-84, 101-102
    std::memcpy(out->tau, &tau, 32);
    if (srs_out) {
      *srs_out = nullptr;
      CtxScope g(&ctx->c);
      tns_srs *s = new tns_srs();
      s->s.device = ctx->c.device;
      s->s.n = out->num_powers;
      s->s.has_tau = true;
      s->s.tau = tau;
      try {
        G1Affine *pts = (G1Affine *)s->s.points.ensure(sizeof(G1Affine) * s->s.n);
        srs_generate_dev(&ctx->c, tau, s->s.n, pts);
      } catch (...) {
        delete s;
        throw;
      }
      *srs_out = s;
    }
    return TNS_OK;
  });
}

int tns_srs_upload(tns_ctx *ctx, const uint64_t *g1, size_t n, tns_srs **out) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    tns_srs *s = new tns_srs();
    s->s.device = ctx->c.device;
    s->s.n = n;
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
    if (n > srs->s.n) throw Error(TNS_ERR_INVALID_PARAMETERS, "download beyond SRS length");
    if (n) TNS_HIP(hipMemcpy(g1_out, srs->s.points.p, sizeof(G1Affine) * n, hipMemcpyDeviceToHost));
    return TNS_OK;
  });
}

size_t tns_srs_len(const tns_srs *srs) { return srs ? srs->s.n : 0; }

int tns_srs_set_tau(tns_srs *srs, const uint64_t tau[4]) {
  return guarded([&]() {
    if (!srs) throw Error(TNS_ERR_INVALID_PARAMETERS, "null SRS");
    Fr t;
    std::memcpy(&t, tau, 32);
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
    const LagrangeBasis *b = lagrange_basis_dev(&ctx->c, srs->s, n);
    ctx->c.lagrange_commit = saved;
    (void)b;  // nullptr only when tau is itself a node: the coefficient path is used then
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
  if (n == 0 || (n & (n - 1))) throw Error(TNS_ERR_POLYNOMIAL, "evaluation vector length must be a power of two");
  Fr *dy = (Fr *)d.ensure(sizeof(Fr) * n);
  TNS_HIP(hipMemcpyAsync(dy, evals, sizeof(Fr) * n, hipMemcpyHostToDevice, ctx->c.stream));
  p.y = dy;
  p.N = n;
  p.coeffs = (Fr *)cf.ensure(sizeof(Fr) * n);
}

int tns_kzg_commit_evals(tns_ctx *ctx, const tns_srs *srs, const uint64_t *evals, size_t n, uint64_t out[12]) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    DevBuf d, cf;
    EvalPoly p;
    upload_evals(ctx, evals, n, d, cf, p);
    store_proj(commit_evals(&ctx->c, srs->s, p), out);
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
    p.basis = lagrange_basis_dev(&ctx->c, srs->s, n);
    Fr zz, v;
    std::memcpy(&zz, z, 32);
    G1Affine pi;
    open_evals(&ctx->c, srs->s, p, zz, &v, &pi, s);
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

int tns_mle_evaluate(tns_ctx *ctx, const uint64_t *evals, unsigned nv, const uint64_t *point, uint64_t out[4]) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    if (nv > 30) throw Error(TNS_ERR_INVALID_PARAMETERS, "too many variables");
    size_t n = (size_t)1 << nv;
    DevBuf d;
    Fr *pe = (Fr *)d.ensure(sizeof(Fr) * n);
    TNS_HIP(hipMemcpyAsync(pe, evals, sizeof(Fr) * n, hipMemcpyHostToDevice, ctx->c.stream));
    std::vector<Fr> pt(nv ? nv : 1);
    if (nv) std::memcpy(pt.data(), point, 32 * (size_t)nv);
    Fr r = mle_evaluate_dev(&ctx->c, pe, nv, pt.data());
    std::memcpy(out, &r, 32);
    return TNS_OK;
  });
}

int tns_mle_partial_evaluate(tns_ctx *ctx, const uint64_t *evals, unsigned nv, const uint64_t *fixed,
                             unsigned k, uint64_t *out) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    if (k > nv) throw Error(TNS_ERR_INVALID_PARAMETERS, "Cannot fix more variables than available");
    size_t n = (size_t)1 << nv;
    DevBuf a, b;
    Fr *pa = (Fr *)a.ensure(sizeof(Fr) * n), *pb = (Fr *)b.ensure(sizeof(Fr) * (n / 2 + 1));
    TNS_HIP(hipMemcpyAsync(pa, evals, sizeof(Fr) * n, hipMemcpyHostToDevice, ctx->c.stream));
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

int tns_sumcheck_prove(tns_ctx *ctx, const uint64_t *const *tables, int n_tables, unsigned nv,
                       const uint64_t claimed[4], const tns_term *terms, int n_terms, tns_transcript *tr,
                       uint64_t *rounds_out, uint64_t final_out[4], uint64_t *challenges_out) {
  return guarded([&]() {
    CtxScope g(&ctx->c);
    if (nv > 30 || n_tables < 0 || n_tables > 4)
      throw Error(TNS_ERR_INVALID_PARAMETERS, "unsupported sum-check shape (<= 4 tables)");
    size_t n = (size_t)1 << nv;
    std::vector<DevBuf> bufs(n_tables);
    std::vector<Fr *> ptrs(n_tables);
    for (int i = 0; i < n_tables; i++) {
      ptrs[i] = (Fr *)bufs[i].ensure(sizeof(Fr) * n);
      TNS_HIP(hipMemcpyAsync(ptrs[i], tables[i], sizeof(Fr) * n, hipMemcpyHostToDevice, ctx->c.stream));
    }
    std::vector<SumcheckTerm> st(n_terms);
    for (int t = 0; t < n_terms; t++) {
      std::memcpy(&st[t].coeff, terms[t].coeff, 32);
      for (int j = 0; j < 3; j++) st[t].tab[j] = terms[t].tables[j];
    }
    Fr cl;
    std::memcpy(&cl, claimed, 32);
    std::vector<Fr> rounds(4 * (size_t)(nv ? nv : 1)), chal(nv ? nv : 1);
    Fr finals[4], fe;
    int rc = sumcheck_prove_dev(&ctx->c, ptrs.data(), n_tables, nv, cl, st.data(), n_terms, tr->t,
                                rounds.data(), chal.data(), finals, &fe);
    std::memcpy(rounds_out, rounds.data(), 128 * (size_t)nv);
    if (challenges_out) std::memcpy(challenges_out, chal.data(), 32 * (size_t)nv);
    std::memcpy(final_out, &fe, 32);
    return rc;
  });
}

int tns_last_prove_timing(tns_ctx *ctx, double out_ms[6]) {
  for (int i = 0; i < 6; i++) out_ms[i] = ctx->timing[i];
  return TNS_OK;
}

// ---------------------------------------------------------------- protocols
static void fill_common_tail(Ctx *c, const Srs &srs, HostTranscript &tr, Fr *const *mles, int n_mles,
                             unsigned nv, EvalPoly &polyA, EvalPoly &polyB, tns_proof *out, double *timing,
                             DevBuf &sbuf) {
  Timer t_sc;
  std::vector<Fr> rounds(4 * (size_t)(nv ? nv : 1)), chal(nv ? nv : 1);
  Fr finals[4], fe;
  // zero constraint closure (src/twist.rs:186-214, src/shout.rs:160-184): no terms
  sumcheck_prove_dev(c, mles, n_mles, nv, Fr::zero(), nullptr, 0, tr, rounds.data(), chal.data(), finals, &fe);
  out->num_rounds = nv;
  std::memcpy(out->round_polynomials, rounds.data(), 128 * (size_t)nv);
  std::memcpy(out->sumcheck_challenges, chal.data(), 32 * (size_t)nv);
  std::memcpy(out->final_evaluation, &fe, 32);
  for (int i = 0; i < n_mles && i < 3; i++) std::memcpy(out->final_mle_evals[i], &finals[i], 32);
  timing[3] = t_sc.ms();
  // challenge_field_elements("opening_challenges", nv) (src/utils.rs:195-203); only [0] used
  Timer t_open;
  if (nv >= 1) {
    Fr z = tr.challenge("opening_challenges_0");
    char lab[64];
    for (unsigned i = 1; i < nv; i++) {
      snprintf(lab, sizeof lab, "opening_challenges_%u", i);
      (void)tr.challenge(lab);
    }
    std::memcpy(out->opening_point, &z, 32);
    Fr va, vb;
    G1Affine pa, pb;
    open_evals(c, srs, polyA, z, &va, &pa, sbuf);
    open_evals(c, srs, polyB, z, &vb, &pb, sbuf);
    store_proj(pa, out->opening_proofs[0]);
    store_proj(pb, out->opening_proofs[1]);
    std::memcpy(out->final_evaluations[0], &va, 32);
    std::memcpy(out->final_evaluations[1], &vb, 32);
    out->num_openings = 2;
  }
  timing[4] = t_open.ms();
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

// Twist::prove (src/twist.rs:107-252).  kind: where addr/value/is_write live (H2D or D2D).
static void twist_core(tns_ctx *ctx, const tns_srs *srs, const tns_params *params, const uint64_t *addr,
                       const uint64_t *value, const uint8_t *is_write, size_t n_ops, tns_proof *out,
                       hipMemcpyKind kind) {
  Timer total;
  CtxScope g(&ctx->c);
  Ctx *c = &ctx->c;
  hipStream_t st = c->stream;
  std::memset(out, 0, sizeof *out);
  if (n_ops > params->max_operations)  // src/twist.rs:108-112
    throw Error(TNS_ERR_INVALID_PARAMETERS, "Too many operations");
  const size_t N = next_pow2(n_ops);  // :141 next_power_of_two().max(1)
  const unsigned nv = ilog2_exact(N);
  if (nv > TNS_MAX_ROUNDS) throw Error(TNS_ERR_INVALID_PARAMETERS, "trace too long");
  double *tm = ctx->timing;
  for (int i = 0; i < 6; i++) tm[i] = 0;
  // ---- SoA extraction / padding into the resident workspace (src/twist.rs:115-148)
  Timer t_h2d;
  DevBuf &d_addr_raw = c->prove_ws[0], &d_flags = c->prove_ws[1], &d_a = c->prove_ws[2],
         &d_v = c->prove_ws[3], &d_o = c->prove_ws[4], &d_ca = c->prove_ws[5], &d_cv = c->prove_ws[6],
         &d_s = c->prove_ws[7];
  Fr *A = (Fr *)d_a.ensure(sizeof(Fr) * N), *V = (Fr *)d_v.ensure(sizeof(Fr) * N), *O = (Fr *)d_o.ensure(sizeof(Fr) * N);
  const uint64_t *ar = addr;
  const uint8_t *fl = is_write;
  if (kind == hipMemcpyHostToDevice) {
    uint64_t *dar = (uint64_t *)d_addr_raw.ensure(8 * (n_ops ? n_ops : 1));
    uint8_t *dfl = (uint8_t *)d_flags.ensure(n_ops ? n_ops : 1);
    if (n_ops) {
      TNS_HIP(hipMemcpyAsync(dar, addr, 8 * n_ops, hipMemcpyHostToDevice, st));
      TNS_HIP(hipMemcpyAsync(dfl, is_write, n_ops, hipMemcpyHostToDevice, st));
    }
    ar = dar;
    fl = dfl;
  }
  if (n_ops) TNS_HIP(hipMemcpyAsync(V, value, sizeof(Fr) * n_ops, kind, st));
  fr_fill_zero_dev(c, A, N);
  to_mont_u64_dev(c, ar, A, n_ops);
  if (N > n_ops) fr_fill_zero_dev(c, V + n_ops, N - n_ops);
  k_write_flags<<<grid_for(N, 256), 256, 0, st>>>(fl, O, n_ops, N);
  TNS_LAUNCH_CHECK();
  TNS_HIP(hipStreamSynchronize(st));
  tm[0] = t_h2d.ms();
  // ---- vector_to_polynomial + commit x2 (src/twist.rs:151-163).  The sum-check below
  // folds A and V in place, so the openings work from copies of the evaluations.
  Timer t_int;
  EvalPoly pa, pv;
  pa.N = pv.N = N;
  pa.coeffs = (Fr *)d_ca.ensure(sizeof(Fr) * N);
  pv.coeffs = (Fr *)d_cv.ensure(sizeof(Fr) * N);
  Fr *YA = (Fr *)c->prove_ws[8].ensure(sizeof(Fr) * N), *YV = (Fr *)c->prove_ws[9].ensure(sizeof(Fr) * N);
  TNS_HIP(hipMemcpyAsync(YA, A, sizeof(Fr) * N, hipMemcpyDeviceToDevice, st));
  TNS_HIP(hipMemcpyAsync(YV, V, sizeof(Fr) * N, hipMemcpyDeviceToDevice, st));
  pa.y = YA;
  pv.y = YV;
  tm[1] = t_int.ms();
  Timer t_com;
  G1Affine Ca = commit_evals(c, srs->s, pa);
  G1Affine Cv = commit_evals(c, srs->s, pv);
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
  fill_common_tail(c, srs->s, tr, mles, 3, nv, pa, pv, out, tm, d_s);
  TNS_HIP(hipStreamSynchronize(st));
  tm[5] = total.ms();
}

int tns_twist_prove(tns_ctx *ctx, const tns_srs *srs, const tns_params *params, const uint64_t *addr,
                    const uint64_t *value, const uint8_t *is_write, size_t n_ops, tns_proof *out) {
  return guarded([&]() {
    twist_core(ctx, srs, params, addr, value, is_write, n_ops, out, hipMemcpyHostToDevice);
    return TNS_OK;
  });
}

int tns_twist_prove_device(tns_ctx *ctx, const tns_srs *srs, const tns_params *params, const uint64_t *d_addr,
                           const uint64_t *d_value, const uint8_t *d_is_write, size_t n_ops, tns_proof *out) {
  return guarded([&]() {
    twist_core(ctx, srs, params, d_addr, d_value, d_is_write, n_ops, out, hipMemcpyDeviceToDevice);
    return TNS_OK;
  });
}

// Shout::prove (src/shout.rs:97-222)
static void shout_core(tns_ctx *ctx, const tns_srs *srs, const tns_params *params, const uint64_t *entries,
                       size_t n_entries, const uint64_t *indices, size_t n_lookups, tns_proof *out,
                       hipMemcpyKind kind) {
  Timer total;
  CtxScope g(&ctx->c);
  Ctx *c = &ctx->c;
  hipStream_t st = c->stream;
  std::memset(out, 0, sizeof *out);
  if (n_lookups > params->max_operations)  // src/shout.rs:98-102
    throw Error(TNS_ERR_INVALID_PARAMETERS, "Too many lookup operations");
  const size_t T = next_pow2(n_entries), M = next_pow2(n_lookups);  // :105, :116
  const unsigned nv = ilog2_exact(M);
  if (nv > TNS_MAX_ROUNDS) throw Error(TNS_ERR_INVALID_PARAMETERS, "too many lookups");
  double *tm = ctx->timing;
  for (int i = 0; i < 6; i++) tm[i] = 0;
  Timer t_h2d;
  DevBuf &d_idx_raw = c->prove_ws[0], &d_bad = c->prove_ws[1], &d_t = c->prove_ws[2], &d_i = c->prove_ws[3],
         &d_ct = c->prove_ws[5], &d_ci = c->prove_ws[6], &d_s = c->prove_ws[7];
  Fr *TB = (Fr *)d_t.ensure(sizeof(Fr) * T), *I = (Fr *)d_i.ensure(sizeof(Fr) * M);
  fr_fill_zero_dev(c, TB, T);
  fr_fill_zero_dev(c, I, M);
  if (n_entries) TNS_HIP(hipMemcpyAsync(TB, entries, sizeof(Fr) * n_entries, kind, st));
  if (n_lookups) {
    const uint64_t *ir = indices;
    if (kind == hipMemcpyHostToDevice) {
      uint64_t *dir = (uint64_t *)d_idx_raw.ensure(8 * n_lookups);
      TNS_HIP(hipMemcpyAsync(dir, indices, 8 * n_lookups, hipMemcpyHostToDevice, st));
      ir = dir;
    }
    // LookupTable::lookup bounds (src/shout.rs:44-50)
    unsigned *bad = (unsigned *)d_bad.ensure(sizeof(unsigned));
    TNS_HIP(hipMemsetAsync(bad, 0, sizeof(unsigned), st));
    k_max_index_check<<<grid_for(n_lookups, 256), 256, 0, st>>>(ir, n_lookups, n_entries, bad);
    TNS_LAUNCH_CHECK();
    unsigned hbad = 0;
    TNS_HIP(hipMemcpyAsync(&hbad, bad, sizeof hbad, hipMemcpyDeviceToHost, st));
    TNS_HIP(hipStreamSynchronize(st));
    if (hbad) throw Error(TNS_ERR_INVALID_PARAMETERS, "Lookup index out of bounds");
    to_mont_u64_dev(c, ir, I, n_lookups);
  }
  TNS_HIP(hipStreamSynchronize(st));
  tm[0] = t_h2d.ms();
  Timer t_int;
  EvalPoly pt, pi;
  pt.N = T;
  pi.N = M;
  pt.coeffs = (Fr *)d_ct.ensure(sizeof(Fr) * T);
  pi.coeffs = (Fr *)d_ci.ensure(sizeof(Fr) * M);
  Fr *YI = (Fr *)c->prove_ws[8].ensure(sizeof(Fr) * M);  // the sum-check folds I in place
  TNS_HIP(hipMemcpyAsync(YI, I, sizeof(Fr) * M, hipMemcpyDeviceToDevice, st));
  pt.y = TB;
  pi.y = YI;
  tm[1] = t_int.ms();
  Timer t_com;
  G1Affine Ct = commit_evals(c, srs->s, pt);  // table first (src/shout.rs:125-133)
  G1Affine Ci = commit_evals(c, srs->s, pi);
  store_proj(Ct, out->commitments[0]);
  store_proj(Ci, out->commitments[1]);
  tm[2] = t_com.ms();
  HostTranscript tr;
  tr.append_label("table_commitment");
  tr.append_fr(commitment_hash(Ct));
  tr.append_label("index_commitment");
  tr.append_fr(commitment_hash(Ci));
  Fr *mles[1] = {I};  // the closure evaluates only the index MLE (src/shout.rs:175)
  fill_common_tail(c, srs->s, tr, mles, 1, nv, pt, pi, out, tm, d_s);
  TNS_HIP(hipStreamSynchronize(st));
  tm[5] = total.ms();
}

int tns_shout_prove(tns_ctx *ctx, const tns_srs *srs, const tns_params *params, const uint64_t *entries,
                    size_t n_entries, const uint64_t *indices, size_t n_lookups, tns_proof *out) {
  return guarded([&]() {
    shout_core(ctx, srs, params, entries, n_entries, indices, n_lookups, out, hipMemcpyHostToDevice);
    return TNS_OK;
  });
}

int tns_shout_prove_device(tns_ctx *ctx, const tns_srs *srs, const tns_params *params, const uint64_t *d_entries,
                           size_t n_entries, const uint64_t *d_indices, size_t n_lookups, tns_proof *out) {
  return guarded([&]() {
    shout_core(ctx, srs, params, d_entries, n_entries, d_indices, n_lookups, out, hipMemcpyDeviceToDevice);
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

// ---------------------------------------------------------------- kernel timing (HIP events)
int tns_profile_enable(tns_ctx *ctx, int on) {
  ctx->c.prof.enabled = on != 0;
  ctx->c.prof.reset();
  return TNS_OK;
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

int tns_bench_trace(size_t memory_size, size_t n_ops, uint64_t *addr, uint64_t *value, uint8_t *is_write) {
  return guarded([&]() {
    if (memory_size == 0 || (memory_size & (memory_size - 1)))
      throw Error(TNS_ERR_INVALID_PARAMETERS, "Memory size must be power of 2");
    std::vector<uint64_t> mem(memory_size, 0);
    for (size_t i = 0; i < n_ops; i++) {
      if (i % 3 == 0) {
        size_t a = i % memory_size;
        mem[a] = (uint64_t)i * 42;
        addr[i] = a;
        value[i] = mem[a];
        is_write[i] = 1;
      } else {
        size_t a = (i / 2) % memory_size;
        addr[i] = a;
        value[i] = mem[a];
        is_write[i] = 0;
      }
    }
    return TNS_OK;
  });
}

}  // extern "C"
