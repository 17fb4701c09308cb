/*
 * fastcpu.c -- the "fast CPU" baseline of SURVEY.md 8(d): Twist::prove (src/twist.rs:107-252)
 * with the SAME algorithms as the MI355X path, on host threads:
 *   - KZG in the Lagrange basis of the nodes 0..N-1 (commit = MSM over [L_j(tau)]G, the
 *     setup-time basis; src/commitments.rs:162-180 applied to vector_to_polynomial(v)),
 *   - barycentric opening at z and the quotient's node values (src/commitments.rs:182-199),
 *   - the zero-closure sum-check as table folds (src/sumcheck.rs:56-110),
 *   - Pippenger MSM (unsigned c-bit windows, per-task Jacobian buckets, running sums).
 * BASELINE / TEST INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg times it, tests pin it to
 * the reference-algorithm restatement (oracle.c).  Never part of the product path.
 *
 * Unity build: liboracle.so is this file, which includes oracle.c, so both share one copy of
 * the field, curve and transcript code (4 x u64 limbs, unsigned __int128).
 */
#include "oracle.c"

#include <pthread.h>

#include "fastcpu.h"

/* ------------------------------------------------------------- par-for over host threads */
typedef void (*range_fn)(void *ctx, size_t a, size_t b, int tid);
typedef struct {
  range_fn f;
  void *ctx;
  size_t a, b;
  int tid;
} fc_job;

static void *fc_run(void *p) {
  fc_job *j = (fc_job *)p;
  if (j->a < j->b) j->f(j->ctx, j->a, j->b, j->tid);
  return NULL;
}

#define FC_MAX_THREADS 256
/* [0, n) in T contiguous ranges, range t on thread t (t = 0 on the caller) */
static void par_for(size_t n, int T, range_fn f, void *ctx) {
  if (T < 1) T = 1;
  if (T > FC_MAX_THREADS) T = FC_MAX_THREADS;
  pthread_t th[FC_MAX_THREADS];
  fc_job jb[FC_MAX_THREADS];
  size_t per = (n + T - 1) / T;
  for (int t = 0; t < T; t++) {
    size_t a = (size_t)t * per, b = a + per;
    jb[t] = (fc_job){f, ctx, a < n ? a : n, b < n ? b : n, t};
  }
  for (int t = 1; t < T; t++) pthread_create(&th[t], NULL, fc_run, &jb[t]);
  fc_run(&jb[0]);
  for (int t = 1; t < T; t++) pthread_join(th[t], NULL);
}

/* ------------------------------------------------------------- mixed addition */
/* madd-2007-bl: Jacobian + affine (affine identity = all zero words) */
static void jac_madd(jac *r, const jac *p, const u64 *q) {
  if (is_zero4(q) && is_zero4(q + 4)) { *r = *p; return; }
  if (is_zero4(p->z)) { aff_to_jac(r, q); return; }
  u64 Z1Z1[4], U2[4], S2[4], H[4], HH[4], I[4], J[4], rr[4], V[4], t[4];
  jac o;
  fmul(&FQ, Z1Z1, p->z, p->z);
  fmul(&FQ, U2, q, Z1Z1);
  fmul(&FQ, S2, q + 4, p->z);
  fmul(&FQ, S2, S2, Z1Z1);
  fsub(&FQ, H, U2, p->x);
  fsub(&FQ, rr, S2, p->y);
  if (is_zero4(H)) {
    if (is_zero4(rr)) {
      jac qj;
      aff_to_jac(&qj, q);
      jac_dbl(r, &qj);
    } else {
      jac_zero(r);
    }
    return;
  }
  fadd(&FQ, rr, rr, rr);
  fmul(&FQ, HH, H, H);
  fadd(&FQ, I, HH, HH);
  fadd(&FQ, I, I, I);
  fmul(&FQ, J, H, I);
  fmul(&FQ, V, p->x, I);
  fmul(&FQ, o.x, rr, rr);
  fsub(&FQ, o.x, o.x, J);
  fsub(&FQ, o.x, o.x, V);
  fsub(&FQ, o.x, o.x, V);
  fsub(&FQ, t, V, o.x);
  fmul(&FQ, o.y, rr, t);
  fmul(&FQ, t, p->y, J);
  fadd(&FQ, t, t, t);
  fsub(&FQ, o.y, o.y, t);
  fadd(&FQ, t, p->z, H);
  fmul(&FQ, t, t, t);
  fsub(&FQ, t, t, Z1Z1);
  fsub(&FQ, o.z, t, HH);
  *r = o;
}

/* ------------------------------------------------------------- Pippenger MSM */
typedef struct {
  const u64 *pts; /* affine, n x 8 */
  const u64 *k;   /* canonical scalars, n x 4 */
  size_t n;
  int c, W, tpw; /* window bits, windows, point ranges per window */
  jac *part;     /* one partial window sum per task */
} msm_job;

static unsigned digit(const u64 k[4], int bit, int c) {
  int w = bit >> 6, s = bit & 63;
  u64 lo = w < 4 ? k[w] >> s : 0;
  if (s && w + 1 < 4) lo |= k[w + 1] << (64 - s);
  return (unsigned)(lo & ((1ULL << c) - 1));
}

static void msm_tasks(void *vctx, size_t a, size_t b, int tid) {
  msm_job *J = (msm_job *)vctx;
  const size_t nb = ((size_t)1 << J->c) - 1;
  jac *B = (jac *)malloc(nb * sizeof(jac));
  for (size_t task = a; task < b; task++) {
    const int w = (int)(task / J->tpw), r = (int)(task % J->tpw);
    const size_t lo = J->n * r / J->tpw, hi = J->n * (r + 1) / J->tpw;
    for (size_t j = 0; j < nb; j++) jac_zero(&B[j]);
    for (size_t i = lo; i < hi; i++) {
      unsigned d = digit(J->k + 4 * i, w * J->c, J->c);
      if (d) jac_madd(&B[d - 1], &B[d - 1], J->pts + 8 * i);
    }
    jac run, acc; /* sum_j (j + 1) B_j by running sums */
    jac_zero(&run);
    jac_zero(&acc);
    for (size_t j = nb; j-- > 0;) {
      jac_add(&run, &run, &B[j]);
      jac_add(&acc, &acc, &run);
    }
    J->part[task] = acc;
  }
  free(B);
  (void)tid;
}

typedef struct {
  const u64 *in;
  u64 *out;
} canon_job;
static void canon_range(void *vctx, size_t a, size_t b, int tid) {
  canon_job *J = (canon_job *)vctx;
  for (size_t i = a; i < b; i++) from_mont(&FR, J->out + 4 * i, J->in + 4 * i);
  (void)tid;
}

/* sum_i s_i P_i: affine points (n x 8), Montgomery scalars (n x 4); result affine */
static void fc_msm(const u64 *pts, const u64 *scal, size_t n, int T, u64 out[8]) {
  u64 *k = (u64 *)malloc((n ? n : 1) * 32);
  canon_job cj = {scal, k};
  par_for(n, T, canon_range, &cj);
  int bits = 0;
  for (size_t i = 0; i < n; i++)
    for (int l = 3; l >= 0; l--)
      if (k[4 * i + l]) {
        int b = 64 * l + 64 - __builtin_clzll(k[4 * i + l]);
        if (b > bits) bits = b;
        break;
      }
  jac acc;
  jac_zero(&acc);
  if (bits) {
    int lg = 0;
    while (((size_t)1 << lg) < n) lg++;
    int c = lg > 6 ? lg - 4 : 2; /* ~n/16 buckets per window: the running sums stay minor */
    if (c > 16) c = 16;
    const int W = (bits + c - 1) / c;
    int tpw = (T + W - 1) / W;
    if ((size_t)tpw > n) tpw = (int)n;
    msm_job J = {pts, k, n, c, W, tpw, (jac *)malloc(sizeof(jac) * W * tpw)};
    par_for((size_t)W * tpw, T, msm_tasks, &J);
    for (int w = W - 1; w >= 0; w--) {
      for (int s = 0; s < c; s++) jac_dbl(&acc, &acc);
      for (int r = 0; r < tpw; r++) jac_add(&acc, &acc, &J.part[(size_t)w * tpw + r]);
    }
    free(J.part);
  }
  free(k);
  jac_to_aff(out, &acc);
}

/* ------------------------------------------------------------- setup-side helpers */
void fc_bary_weights(size_t N, uint64_t *w) {
  u64 *f = (u64 *)malloc(N * 32), *fi = (u64 *)malloc(N * 32);
  memcpy(f, FR.one, 32);
  for (size_t j = 1; j < N; j++) {
    u64 jj[4];
    fr_u64(jj, (u64)j);
    fmul(&FR, f + 4 * j, f + 4 * (j - 1), jj);
  }
  finv(&FR, fi + 4 * (N - 1), f + 4 * (N - 1));
  for (size_t j = N - 1; j > 0; j--) {
    u64 jj[4];
    fr_u64(jj, (u64)j);
    fmul(&FR, fi + 4 * (j - 1), fi + 4 * j, jj);
  }
  for (size_t j = 0; j < N; j++) {
    fmul(&FR, w + 4 * j, fi + 4 * j, fi + 4 * (N - 1 - j));
    if ((N - 1 - j) & 1) fneg(&FR, w + 4 * j, w + 4 * j);
  }
  free(f);
  free(fi);
}

void fc_lagrange_basis(const uint64_t tau[4], size_t N, uint64_t *out) {
  u64 *w = (u64 *)malloc(N * 32);
  fc_bary_weights(N, w);
  u64 ell[4];
  memcpy(ell, FR.one, 32);
  for (size_t j = 0; j < N; j++) {
    u64 d[4], jj[4];
    fr_u64(jj, (u64)j);
    fsub(&FR, d, tau, jj);
    fmul(&FR, ell, ell, d);
  }
  jac gen;
  u64 gaff[8] = {0};
  u64 one_c[4] = {1, 0, 0, 0}, two_c[4] = {2, 0, 0, 0};
  to_mont(&FQ, gaff, one_c);
  to_mont(&FQ, gaff + 4, two_c);
  aff_to_jac(&gen, gaff);
  for (size_t j = 0; j < N; j++) { /* L_j(tau) = ell(tau) w_j / (tau - j) */
    u64 d[4], jj[4], s[4];
    fr_u64(jj, (u64)j);
    fsub(&FR, d, tau, jj);
    finv(&FR, d, d);
    fmul(&FR, s, ell, w + 4 * j);
    fmul(&FR, s, s, d);
    jac P;
    jac_mul(&P, &gen, s);
    jac_to_aff(out + 8 * j, &P);
  }
  free(w);
}

/* ------------------------------------------------------------- Twist::prove */
typedef struct {
  const uint64_t *addr, *val;
  const uint8_t *isw;
  size_t n_ops;
  u64 *A, *V, *O;
} soa_job;
static void soa_range(void *vctx, size_t a, size_t b, int tid) {
  soa_job *J = (soa_job *)vctx;
  for (size_t i = a; i < b; i++) { /* SoA extraction + zero padding (src/twist.rs:115-148) */
    if (i < J->n_ops) {
      fr_u64(J->A + 4 * i, J->addr[i]);
      memcpy(J->V + 4 * i, J->val + 4 * i, 32);
      if (J->isw[i]) memcpy(J->O + 4 * i, FR.one, 32);
      else memset(J->O + 4 * i, 0, 32);
    } else {
      memset(J->A + 4 * i, 0, 32);
      memset(J->V + 4 * i, 0, 32);
      memset(J->O + 4 * i, 0, 32);
    }
  }
  (void)tid;
}

typedef struct {
  u64 *T[3];
  const u64 *r;
  u64 *tmp[3];
} fold_job;
static void fold_range(void *vctx, size_t a, size_t b, int tid) {
  fold_job *J = (fold_job *)vctx;
  for (int t = 0; t < 3; t++)
    for (size_t s = a; s < b; s++) { /* T'[s] = T[2s] + r (T[2s+1] - T[2s]) (src/polynomials.rs:111-119) */
      u64 d[4];
      fsub(&FR, d, J->T[t] + 8 * s + 4, J->T[t] + 8 * s);
      fmul(&FR, d, d, J->r);
      fadd(&FR, J->tmp[t] + 4 * s, J->T[t] + 8 * s, d);
    }
  (void)tid;
}

typedef struct {
  const u64 *z, *w, *y0, *y1;
  u64 *inv;           /* 1 / (z - j) */
  u64 *ell, *s0, *s1; /* per range: prod (z - j), sum w_j y_j / (z - j) */
  int bad;
} bary_job;
static void bary_range(void *vctx, size_t a, size_t b, int tid) {
  bary_job *J = (bary_job *)vctx;
  u64 acc[4], jj[4], d[4];
  memcpy(acc, FR.one, 32);
  for (size_t j = a; j < b; j++) { /* Montgomery batch inversion over the range */
    fr_u64(jj, (u64)j);
    fsub(&FR, d, J->z, jj);
    if (is_zero4(d)) J->bad = 1;
    memcpy(J->inv + 4 * j, acc, 32);
    fmul(&FR, acc, acc, d);
  }
  memcpy(J->ell + 4 * tid, acc, 32);
  u64 iv[4];
  finv(&FR, iv, acc);
  u64 s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0};
  for (size_t j = b; j-- > a;) {
    fr_u64(jj, (u64)j);
    fsub(&FR, d, J->z, jj);
    u64 ij[4], t[4];
    fmul(&FR, ij, iv, J->inv + 4 * j);
    fmul(&FR, iv, iv, d);
    memcpy(J->inv + 4 * j, ij, 32);
    fmul(&FR, ij, ij, J->w + 4 * j);
    fmul(&FR, t, ij, J->y0 + 4 * j);
    fadd(&FR, s0, s0, t);
    fmul(&FR, t, ij, J->y1 + 4 * j);
    fadd(&FR, s1, s1, t);
  }
  memcpy(J->s0 + 4 * tid, s0, 32);
  memcpy(J->s1 + 4 * tid, s1, 32);
}

/* f0(x), f1(x) of two evaluation vectors on the nodes 0..N-1 (y0 / y1: N x 4 Montgomery, y1 may
 * equal y0), ell(x) = prod_j (x - j) and, when inv != NULL, inv[j] = 1 / (x - j): the barycentric
 * form f(x) = ell(x) sum_j w_j y_j / (x - j) in O(N) (one batch inversion per thread range).
 * Returns 1 when x is a node (outputs undefined), else 0. */
static int bary_pair(const u64 *w, const u64 *y0, const u64 *y1, size_t N, const u64 x[4], int T, u64 *inv,
                     u64 f0[4], u64 f1[4], u64 ell_out[4]) {
  u64 *own = inv ? NULL : (u64 *)malloc(N * 32);
  u64 *parts = (u64 *)calloc(3 * (size_t)T, 32);
  bary_job bj = {x, w, y0, y1, inv ? inv : own, parts, parts + 4 * T, parts + 8 * T, 0};
  par_for(N, T, bary_range, &bj);
  u64 ell[4], s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0};
  memcpy(ell, FR.one, 32);
  for (int t = 0; t < T; t++) {
    if (is_zero4(parts + 4 * t)) continue; /* a range no thread ran (ell parts are non-zero) */
    fmul(&FR, ell, ell, parts + 4 * t);
    fadd(&FR, s0, s0, parts + 4 * (T + t));
    fadd(&FR, s1, s1, parts + 4 * (2 * T + t));
  }
  fmul(&FR, f0, ell, s0);
  fmul(&FR, f1, ell, s1);
  if (ell_out) memcpy(ell_out, ell, 32);
  free(parts);
  free(own);
  return bj.bad;
}

int fc_bary_eval2(const uint64_t *bary_w, const uint64_t *y0, const uint64_t *y1, size_t N, const uint64_t x[4],
                  int threads, uint64_t f0[4], uint64_t f1[4], uint64_t ell[4]) {
  const int T = threads < 1 ? 1 : (threads > FC_MAX_THREADS ? FC_MAX_THREADS : threads);
  return bary_pair(bary_w, y0, y1, N, x, T, NULL, f0, f1, ell);
}

void fc_g1_mul_gen(const uint64_t k[4], uint64_t out[8]) {
  u64 gaff[8] = {0};
  u64 one_c[4] = {1, 0, 0, 0}, two_c[4] = {2, 0, 0, 0};
  to_mont(&FQ, gaff, one_c);
  to_mont(&FQ, gaff + 4, two_c);
  jac gen, P;
  aff_to_jac(&gen, gaff);
  jac_mul(&P, &gen, k);
  jac_to_aff(out, &P);
}

void fc_g1_mul(const uint64_t aff[8], const uint64_t k[4], uint64_t out[8]) {
  jac A, P;
  if (is_zero4(aff) && is_zero4(aff + 4)) jac_zero(&A);
  else aff_to_jac(&A, aff);
  jac_mul(&P, &A, k);
  jac_to_aff(out, &P);
}

typedef struct {
  const u64 *y0, *y1, *inv, *v0, *v1;
  u64 *q0, *q1;
} quot_job;
static void quot_range(void *vctx, size_t a, size_t b, int tid) {
  quot_job *J = (quot_job *)vctx;
  for (size_t j = a; j < b; j++) { /* q_j = (P(z) - y_j) / (z - j) */
    u64 d[4];
    fsub(&FR, d, J->v0, J->y0 + 4 * j);
    fmul(&FR, J->q0 + 4 * j, d, J->inv + 4 * j);
    fsub(&FR, d, J->v1, J->y1 + 4 * j);
    fmul(&FR, J->q1 + 4 * j, d, J->inv + 4 * j);
  }
  (void)tid;
}

int fc_twist_prove(const uint64_t *lagrange, const uint64_t *bary_w, size_t N, size_t max_ops,
                   const uint64_t *addr, const uint64_t *val, const uint8_t *is_write, size_t n_ops,
                   int threads, orc_proof *out) {
  memset(out, 0, sizeof *out);
  if (n_ops > max_ops) return 1; /* src/twist.rs:108-112 */
  if (N != next_pow2(n_ops) || N < 2) return 1;
  const int T = threads < 1 ? 1 : (threads > FC_MAX_THREADS ? FC_MAX_THREADS : threads);
  const unsigned nv = log2_exact(N);
  u64 *A = (u64 *)malloc(N * 32), *V = (u64 *)malloc(N * 32), *O = (u64 *)malloc(N * 32);
  u64 *YA = (u64 *)malloc(N * 32), *YV = (u64 *)malloc(N * 32);
  soa_job sj = {addr, val, is_write, n_ops, A, V, O};
  par_for(N, T, soa_range, &sj);
  memcpy(YA, A, N * 32);
  memcpy(YV, V, N * 32);
  /* vector_to_polynomial + commit x2 (src/twist.rs:151-163), in the Lagrange basis */
  fc_msm(lagrange, YA, N, T, out->commitment[0]);
  fc_msm(lagrange, YV, N, T, out->commitment[1]);
  tr_t tr;
  tr_init(&tr);
  u64 h[4];
  orc_commitment_hash(out->commitment[0], h); /* src/twist.rs:170-174 */
  tr_label(&tr, "address_commitment");
  tr_fr(&tr, h);
  orc_commitment_hash(out->commitment[1], h);
  tr_label(&tr, "value_commitment");
  tr_fr(&tr, h);
  /* sum-check of the zero closure: every round polynomial is 0; the tables fold by r */
  out->num_rounds = nv;
  u64 zero[4] = {0, 0, 0, 0};
  u64 *tmp[3] = {(u64 *)malloc(N / 2 * 32), (u64 *)malloc(N / 2 * 32), (u64 *)malloc(N / 2 * 32)};
  u64 *tabs[3] = {A, V, O};
  size_t len = N;
  for (unsigned rnd = 0; rnd < nv; rnd++) {
    char lab[64];
    snprintf(lab, sizeof lab, "sumcheck_round_%u", rnd);
    tr_label(&tr, lab);
    for (int i = 0; i < 4; i++) tr_fr(&tr, zero);
    snprintf(lab, sizeof lab, "sumcheck_challenge_%u", rnd);
    u64 ch[4];
    tr_challenge(&tr, lab, ch);
    memcpy(out->sumcheck_challenges[rnd], ch, 32);
    fold_job fj = {{tabs[0], tabs[1], tabs[2]}, ch, {tmp[0], tmp[1], tmp[2]}};
    par_for(len / 2, T, fold_range, &fj);
    for (int t = 0; t < 3; t++) memcpy(tabs[t], tmp[t], len / 2 * 32);
    len /= 2;
  }
  /* opening challenges (src/utils.rs:195-203); only _0 is used */
  u64 z[4];
  tr_challenge(&tr, "opening_challenges_0", z);
  memcpy(out->opening_point, z, 32);
  for (unsigned i = 1; i < nv; i++) {
    char lab[64];
    u64 dummy[4];
    snprintf(lab, sizeof lab, "opening_challenges_%u", i);
    tr_challenge(&tr, lab, dummy);
  }
  tr_free(&tr);
  /* barycentric values P(z) = ell(z) sum_j w_j y_j / (z - j), quotient node values, MSMs */
  u64 *inv = (u64 *)malloc(N * 32);
  int st = 0;
  if (bary_pair(bary_w, YA, YV, N, z, T, inv, out->final_evaluations[0], out->final_evaluations[1], NULL)) {
    st = 2; /* z on a node (probability ~2^-230): not handled by this baseline */
  } else {
    quot_job qj = {YA, YV, inv, out->final_evaluations[0], out->final_evaluations[1], A, V};
    par_for(N, T, quot_range, &qj);
    fc_msm(lagrange, A, N, T, out->opening_proofs[0]);
    fc_msm(lagrange, V, N, T, out->opening_proofs[1]);
    out->num_openings = 2;
  }
  free(inv);
  for (int t = 0; t < 3; t++) free(tmp[t]);
  free(A);
  free(V);
  free(O);
  free(YA);
  free(YV);
  return st;
}

/* ------------------------------------------------------------- SumCheck::prove, O(N) per round */
/* src/sumcheck.rs:56-110, :156-212 with the closure an MLE composition sum_t c_t prod_j T_{tt[t][j]}
 * (<= 3 factors, <= FC_SC_TABLES tables): instead of evaluating every MLE at every hypercube
 * point (oracle.c sumcheck_core, O(N n) per point), each table is folded once per round
 * (T'[s] = T[2s] + r (T[2s+1] - T[2s]), src/polynomials.rs:111-119) and round k sums the
 * composition of the values T_k[2s] + X (T_k[2s+1] - T_k[2s]) at X = 0..3.  Same round
 * polynomials, challenges and final evaluation as orc_sumcheck_prove (tests/test_fastcpu.py). */
#define FC_SC_TABLES 4
typedef struct {
  const u64 *src[FC_SC_TABLES];
  u64 *dst[FC_SC_TABLES];
  int k, fold;
  const u64 *r;
  int n_terms;
  const u64 *coeffs;
  const int *tt;
  u64 *part; /* per thread: 4 sums */
} scr_job;

static void sc_round_range(void *vctx, size_t a, size_t b, int tid) {
  scr_job *J = (scr_job *)vctx;
  u64 acc[4][4];
  memset(acc, 0, sizeof acc);
  for (size_t s = a; s < b; s++) {
    u64 f0[FC_SC_TABLES][4], d[FC_SC_TABLES][4];
    for (int i = 0; i < J->k; i++) {
      if (J->fold) {
        const u64 *p = J->src[i] + 16 * s;
        u64 t[4];
        fsub(&FR, t, p + 4, p);
        fmul(&FR, t, t, J->r);
        fadd(&FR, f0[i], p, t);
        fsub(&FR, t, p + 12, p + 8);
        fmul(&FR, t, t, J->r);
        fadd(&FR, d[i], p + 8, t); /* f1 for now */
        memcpy(J->dst[i] + 8 * s, f0[i], 32);
        memcpy(J->dst[i] + 8 * s + 4, d[i], 32);
      } else {
        memcpy(f0[i], J->src[i] + 8 * s, 32);
        memcpy(d[i], J->src[i] + 8 * s + 4, 32);
      }
      fsub(&FR, d[i], d[i], f0[i]);
    }
    u64 v[FC_SC_TABLES][4];
    for (int i = 0; i < J->k; i++) memcpy(v[i], f0[i], 32);
    for (int x = 0; x < 4; x++) {
      if (x)
        for (int i = 0; i < J->k; i++) fadd(&FR, v[i], v[i], d[i]);
      for (int t = 0; t < J->n_terms; t++) {
        u64 p[4];
        memcpy(p, J->coeffs + 4 * t, 32);
        for (int j = 0; j < 3; j++) {
          const int ix = J->tt[3 * t + j];
          if (ix >= 0) fmul(&FR, p, p, v[ix]);
        }
        fadd(&FR, acc[x], acc[x], p);
      }
    }
  }
  memcpy(J->part + 16 * tid, acc, sizeof acc);
}

static void sc_sums(scr_job *J, size_t pairs, int T, u64 e[4][4]) {
  J->part = (u64 *)calloc((size_t)T * 16, 8);
  par_for(pairs, T, sc_round_range, J);
  memset(e, 0, 128);
  for (int t = 0; t < T; t++)
    for (int x = 0; x < 4; x++) fadd(&FR, e[x], e[x], J->part + 16 * t + 4 * x);
  free(J->part);
}

int fc_sumcheck_prove(const uint64_t *const *tables, int n_tables, unsigned nv, const uint64_t claimed[4],
                      int n_terms, const uint64_t *term_coeffs, const int *term_tables, const uint8_t *prefix,
                      size_t prefix_len, int threads, uint64_t *rounds_out, uint64_t final_out[4],
                      uint64_t *challenges_out) {
  if (n_tables < 0 || n_tables > FC_SC_TABLES || nv > 40) return 1;
  for (int t = 0; t < 3 * n_terms; t++)
    if (term_tables[t] >= n_tables) return 1;
  const int T = threads < 1 ? 1 : (threads > FC_MAX_THREADS ? FC_MAX_THREADS : threads);
  const size_t n = (size_t)1 << nv;
  u64 *buf[2][FC_SC_TABLES];
  for (int i = 0; i < n_tables; i++) {
    buf[0][i] = (u64 *)malloc((n / 2 + 1) * 32);
    buf[1][i] = (u64 *)malloc((n / 4 + 1) * 32);
  }
  tr_t tr;
  tr_init(&tr);
  if (prefix_len) tr_put(&tr, prefix, prefix_len);
  u64 cur[4], r[4] = {0, 0, 0, 0}, xs[4][4];
  memcpy(cur, claimed, 32);
  for (int i = 0; i < 4; i++) fr_u64(xs[i], (u64)i);
  const u64 *src[FC_SC_TABLES];
  for (int i = 0; i < n_tables; i++) src[i] = tables[i];
  int st = 0, pp = 0;
  for (unsigned rnd = 0; rnd < nv; rnd++) {
    scr_job J = {{0}, {0}, n_tables, rnd > 0, r, n_terms, term_coeffs, term_tables, NULL};
    for (int i = 0; i < n_tables; i++) {
      J.src[i] = src[i];
      J.dst[i] = buf[pp][i];
    }
    u64 e[4][4], coeffs[4][4], g0[4], g1[4], sum[4];
    sc_sums(&J, n >> (rnd + 1), T, e);
    if (rnd > 0) {
      for (int i = 0; i < n_tables; i++) src[i] = buf[pp][i];
      pp ^= 1;
    }
    lagrange_points(&xs[0][0], &e[0][0], 4, &coeffs[0][0]); /* src/sumcheck.rs:201-206 */
    horner(&coeffs[0][0], 4, xs[0], g0);
    horner(&coeffs[0][0], 4, xs[1], g1);
    fadd(&FR, sum, g0, g1);
    if (!eq4(sum, cur)) { st = 6; break; } /* src/sumcheck.rs:80-84 */
    memcpy(rounds_out + 16 * rnd, coeffs, 128);
    char lab[64];
    snprintf(lab, sizeof lab, "sumcheck_round_%u", rnd); /* :90-96 */
    tr_label(&tr, lab);
    for (int i = 0; i < 4; i++) tr_fr(&tr, coeffs[i]);
    snprintf(lab, sizeof lab, "sumcheck_challenge_%u", rnd);
    tr_challenge(&tr, lab, r);
    if (challenges_out) memcpy(challenges_out + 4 * rnd, r, 32);
    horner(&coeffs[0][0], 4, r, cur);
  }
  if (!st) { /* bind the last variable; final = the composition at the bound values (:104) */
    u64 vals[FC_SC_TABLES][4];
    for (int i = 0; i < n_tables; i++) {
      if (nv == 0) {
        memcpy(vals[i], src[i], 32);
      } else {
        u64 t[4];
        fsub(&FR, t, src[i] + 4, src[i]);
        fmul(&FR, t, t, r);
        fadd(&FR, vals[i], src[i], t);
      }
    }
    u64 acc[4] = {0, 0, 0, 0};
    for (int t = 0; t < n_terms; t++) {
      u64 p[4];
      memcpy(p, term_coeffs + 4 * t, 32);
      for (int j = 0; j < 3; j++)
        if (term_tables[3 * t + j] >= 0) fmul(&FR, p, p, vals[term_tables[3 * t + j]]);
      fadd(&FR, acc, acc, p);
    }
    memcpy(final_out, acc, 32);
  }
  tr_free(&tr);
  for (int i = 0; i < n_tables; i++) {
    free(buf[0][i]);
    free(buf[1][i]);
  }
  return st;
}

/* sum over the hypercube of the composition (the honest claim of fc_sumcheck_prove) */
typedef struct {
  const u64 *const *tabs;
  int n_terms;
  const u64 *coeffs;
  const int *tt;
  u64 *part;
} csum_job;
static void csum_range(void *vctx, size_t a, size_t b, int tid) {
  csum_job *J = (csum_job *)vctx;
  u64 acc[4] = {0, 0, 0, 0};
  for (size_t s = a; s < b; s++)
    for (int t = 0; t < J->n_terms; t++) {
      u64 p[4];
      memcpy(p, J->coeffs + 4 * t, 32);
      for (int j = 0; j < 3; j++)
        if (J->tt[3 * t + j] >= 0) fmul(&FR, p, p, J->tabs[J->tt[3 * t + j]] + 4 * s);
      fadd(&FR, acc, acc, p);
    }
  memcpy(J->part + 4 * tid, acc, 32);
}

void fc_composition_sum(const uint64_t *const *tables, unsigned nv, int n_terms, const uint64_t *term_coeffs,
                        const int *term_tables, int threads, uint64_t out[4]) {
  const int T = threads < 1 ? 1 : (threads > FC_MAX_THREADS ? FC_MAX_THREADS : threads);
  csum_job J = {tables, n_terms, term_coeffs, term_tables, (u64 *)calloc((size_t)T * 4, 8)};
  par_for((size_t)1 << nv, T, csum_range, &J);
  u64 s[4] = {0, 0, 0, 0};
  for (int t = 0; t < T; t++) fadd(&FR, s, s, J.part + 4 * t);
  memcpy(out, s, 32);
  free(J.part);
}
