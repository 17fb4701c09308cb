/*
 * oracle.c -- plain-C CPU restatement of the twist-and-shout prover hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Restates, in order:
 *   /root/reference/src/utils.rs:79-204       setup_params, Transcript
 *   /root/reference/src/polynomials.rs:28-161  MultilinearExtension
 *   /root/reference/src/polynomials.rs:301-352 lagrange_interpolate
 *   /root/reference/src/sumcheck.rs:56-212     SumCheck::prove
 *   /root/reference/src/commitments.rs:73-84, 162-199, 305-375  KZG hash/commit/open
 *   /root/reference/src/twist.rs:107-252, src/shout.rs:97-222   prove
 * Third-party semantics (arkworks 0.4.x, rand_chacha 0.3.1, Rust std SipHash-1-3)
 * are restated from their published algorithms; see oracle/pyoracle.py header.
 */
#include "oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef uint64_t u64;

/* ------------------------------------------------------------------ fields */
typedef struct {
  u64 m[4];
  u64 inv;
  u64 one[4];
  u64 r2[4];
} fld;

static const fld FR = {
    {0x43e1f593f0000001ULL, 0x2833e84879b97091ULL, 0xb85045b68181585dULL, 0x30644e72e131a029ULL},
    0xc2e1f593efffffffULL,
    {0xac96341c4ffffffbULL, 0x36fc76959f60cd29ULL, 0x666ea36f7879462eULL, 0x0e0a77c19a07df2fULL},
    {0x1bb8e645ae216da7ULL, 0x53fe3ab1e35c59e3ULL, 0x8c49833d53bb8085ULL, 0x0216d0b17f4e44a5ULL}};
static const fld FQ = {
    {0x3c208c16d87cfd47ULL, 0x97816a916871ca8dULL, 0xb85045b68181585dULL, 0x30644e72e131a029ULL},
    0x87d20782e4866389ULL,
    {0xd35d438dc58f0d9dULL, 0x0a78eb28f5c70b3dULL, 0x666ea36f7879462cULL, 0x0e0a77c19a07df2fULL},
    {0xf32cfc5b538afa89ULL, 0xb5e71911d44501fbULL, 0x47ab1eff0a417ff6ULL, 0x06d89f71cab8351fULL}};

static int geq(const u64 a[4], const u64 b[4]) {
  for (int i = 3; i >= 0; i--) {
    if (a[i] > b[i]) return 1;
    if (a[i] < b[i]) return 0;
  }
  return 1;
}
static u64 sub4(u64 r[4], const u64 a[4], const u64 b[4]) {
  u64 br = 0;
  for (int i = 0; i < 4; i++) {
    u128 d = (u128)a[i] - b[i] - br;
    r[i] = (u64)d;
    br = (u64)(d >> 64) & 1;
  }
  return br;
}
static u64 add4(u64 r[4], const u64 a[4], const u64 b[4]) {
  u64 c = 0;
  for (int i = 0; i < 4; i++) {
    u128 s = (u128)a[i] + b[i] + c;
    r[i] = (u64)s;
    c = (u64)(s >> 64);
  }
  return c;
}
static int is_zero4(const u64 a[4]) { return !(a[0] | a[1] | a[2] | a[3]); }
static int eq4(const u64 a[4], const u64 b[4]) {
  return a[0] == b[0] && a[1] == b[1] && a[2] == b[2] && a[3] == b[3];
}
static void fadd(const fld *F, u64 r[4], const u64 a[4], const u64 b[4]) {
  u64 t[4];
  add4(t, a, b);
  if (geq(t, F->m)) sub4(t, t, F->m);
  memcpy(r, t, 32);
}
static void fsub(const fld *F, u64 r[4], const u64 a[4], const u64 b[4]) {
  u64 t[4];
  if (sub4(t, a, b)) add4(t, t, F->m);
  memcpy(r, t, 32);
}
static void fneg(const fld *F, u64 r[4], const u64 a[4]) {
  if (is_zero4(a)) { memset(r, 0, 32); return; }
  sub4(r, F->m, a);
}
/* CIOS Montgomery multiplication, 64-bit limbs */
static void fmul(const fld *F, u64 r[4], const u64 a[4], const u64 b[4]) {
  u64 t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      c = (u128)a[j] * b[i] + t[j] + (u64)(c >> 64);
      t[j] = (u64)c;
    }
    u128 s = (u128)t[4] + (u64)(c >> 64);
    t[4] = (u64)s;
    t[5] = (u64)(s >> 64);
    u64 m = t[0] * F->inv;
    c = (u128)m * F->m[0] + t[0];
    for (int j = 1; j < 4; j++) {
      c = (u128)m * F->m[j] + t[j] + (u64)(c >> 64);
      t[j - 1] = (u64)c;
    }
    s = (u128)t[4] + (u64)(c >> 64);
    t[3] = (u64)s;
    t[4] = t[5] + (u64)(s >> 64);
  }
  u64 o[4] = {t[0], t[1], t[2], t[3]};
  if (t[4] || geq(o, F->m)) sub4(o, o, F->m);
  memcpy(r, o, 32);
}
static void fpow(const fld *F, u64 r[4], const u64 a[4], const u64 e[4]) {
  u64 acc[4];
  memcpy(acc, F->one, 32);
  for (int i = 255; i >= 0; i--) {
    fmul(F, acc, acc, acc);
    if ((e[i / 64] >> (i % 64)) & 1) fmul(F, acc, acc, a);
  }
  memcpy(r, acc, 32);
}
static void finv(const fld *F, u64 r[4], const u64 a[4]) {
  u64 e[4], two[4] = {2, 0, 0, 0};
  sub4(e, F->m, two);
  fpow(F, r, a, e);
}
static void to_mont(const fld *F, u64 r[4], const u64 a[4]) { fmul(F, r, a, F->r2); }
static void from_mont(const fld *F, u64 r[4], const u64 a[4]) {
  u64 one[4] = {1, 0, 0, 0};
  fmul(F, r, a, one);
}
static void fr_u64(u64 r[4], u64 v) {
  u64 a[4] = {v, 0, 0, 0};
  to_mont(&FR, r, a);
}

void orc_fr_from_u64(uint64_t v, uint64_t out[4]) { fr_u64(out, v); }
void orc_fr_to_canonical(const uint64_t a[4], uint64_t out[4]) { from_mont(&FR, out, a); }
void orc_fr_from_canonical(const uint64_t a[4], uint64_t out[4]) { to_mont(&FR, out, a); }
void orc_fr_mul(const uint64_t a[4], const uint64_t b[4], uint64_t out[4]) { fmul(&FR, out, a, b); }
void orc_fr_inv(const uint64_t a[4], uint64_t out[4]) { finv(&FR, out, a); }

/* ----------------------------------------------------------------- ChaCha20 */
#define ROTL32(v, c) (((v) << (c)) | ((v) >> (32 - (c))))
#define QR(a, b, c, d)                                     \
  x[a] += x[b]; x[d] = ROTL32(x[d] ^ x[a], 16);             \
  x[c] += x[d]; x[b] = ROTL32(x[b] ^ x[c], 12);             \
  x[a] += x[b]; x[d] = ROTL32(x[d] ^ x[a], 8);              \
  x[c] += x[d]; x[b] = ROTL32(x[b] ^ x[c], 7);

void orc_chacha20_block(const uint32_t key[8], uint64_t counter, uint32_t out[16]) {
  uint32_t st[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};
  for (int i = 0; i < 8; i++) st[4 + i] = key[i];
  st[12] = (uint32_t)counter;
  st[13] = (uint32_t)(counter >> 32);
  st[14] = 0;
  st[15] = 0;
  uint32_t x[16];
  memcpy(x, st, sizeof x);
  for (int i = 0; i < 10; i++) {
    QR(0, 4, 8, 12) QR(1, 5, 9, 13) QR(2, 6, 10, 14) QR(3, 7, 11, 15)
    QR(0, 5, 10, 15) QR(1, 6, 11, 12) QR(2, 7, 8, 13) QR(3, 4, 9, 14)
  }
  for (int i = 0; i < 16; i++) out[i] = x[i] + st[i];
}

typedef struct {
  uint32_t key[8];
  u64 counter;
  uint32_t buf[64];
  int idx;
} rng_t;

static void rng_init(rng_t *g, const uint8_t seed[32]) {
  for (int i = 0; i < 8; i++)
    g->key[i] = (uint32_t)seed[4 * i] | ((uint32_t)seed[4 * i + 1] << 8) |
                ((uint32_t)seed[4 * i + 2] << 16) | ((uint32_t)seed[4 * i + 3] << 24);
  g->counter = 0;
  g->idx = 64;
}
static uint32_t rng_u32(rng_t *g) {
  if (g->idx >= 64) { /* rand_chacha 0.3.1 buffers 4 blocks */
    for (int b = 0; b < 4; b++) orc_chacha20_block(g->key, g->counter++, g->buf + 16 * b);
    g->idx = 0;
  }
  return g->buf[g->idx++];
}
static u64 rng_u64(rng_t *g) {
  u64 lo = rng_u32(g);
  u64 hi = rng_u32(g);
  return lo | (hi << 32);
}
/* ark-ff 0.4.2 UniformRand for Fp: limbs are the Montgomery representation */
static void fr_rand(rng_t *g, u64 out[4]) {
  for (;;) {
    u64 l[4];
    for (int i = 0; i < 4; i++) l[i] = rng_u64(g);
    l[3] &= (~0ULL) >> 2;
    if (!geq(l, FR.m)) { memcpy(out, l, 32); return; }
  }
}

/* ----------------------------------------------------------------- SipHash */
#define ROTL64(v, c) (((v) << (c)) | ((v) >> (64 - (c))))
#define SIPROUND                                                         \
  do {                                                                   \
    v0 += v1; v1 = ROTL64(v1, 13); v1 ^= v0; v0 = ROTL64(v0, 32);         \
    v2 += v3; v3 = ROTL64(v3, 16); v3 ^= v2;                             \
    v0 += v3; v3 = ROTL64(v3, 21); v3 ^= v0;                             \
    v2 += v1; v1 = ROTL64(v1, 17); v1 ^= v2; v2 = ROTL64(v2, 32);         \
  } while (0)

uint64_t orc_siphash(const uint8_t *msg, size_t len, uint64_t k0, uint64_t k1, int c, int d) {
  u64 v0 = k0 ^ 0x736f6d6570736575ULL, v1 = k1 ^ 0x646f72616e646f6dULL;
  u64 v2 = k0 ^ 0x6c7967656e657261ULL, v3 = k1 ^ 0x7465646279746573ULL;
  size_t full = len - len % 8;
  for (size_t off = 0; off < full; off += 8) {
    u64 m = 0;
    for (int i = 0; i < 8; i++) m |= (u64)msg[off + i] << (8 * i);
    v3 ^= m;
    for (int i = 0; i < c; i++) SIPROUND;
    v0 ^= m;
  }
  u64 b = ((u64)(len & 0xff)) << 56;
  for (size_t i = full; i < len; i++) b |= (u64)msg[i] << (8 * (i - full));
  v3 ^= b;
  for (int i = 0; i < c; i++) SIPROUND;
  v0 ^= b;
  v2 ^= 0xff;
  for (int i = 0; i < d; i++) SIPROUND;
  return v0 ^ v1 ^ v2 ^ v3;
}

/* --------------------------------------------------------------- Transcript */
typedef struct {
  uint8_t *buf;
  size_t len, cap;
} tr_t;
static void tr_init(tr_t *t) { t->buf = NULL; t->len = t->cap = 0; }
static void tr_free(tr_t *t) { free(t->buf); }
static void tr_put(tr_t *t, const void *p, size_t n) {
  if (t->len + n > t->cap) {
    t->cap = (t->len + n) * 2 + 64;
    t->buf = (uint8_t *)realloc(t->buf, t->cap);
  }
  memcpy(t->buf + t->len, p, n);
  t->len += n;
}
static void tr_label(tr_t *t, const char *s) { tr_put(t, s, strlen(s)); }
static void tr_fr(tr_t *t, const u64 a[4]) { /* compressed Fr: 32 B LE canonical */
  u64 c[4];
  from_mont(&FR, c, a);
  uint8_t b[32];
  for (int i = 0; i < 32; i++) b[i] = (uint8_t)(c[i / 8] >> (8 * (i % 8)));
  tr_put(t, b, 32);
}
/* src/utils.rs:172-192 (state already holds the label) */
static void challenge_from_state(const uint8_t *state, size_t len, u64 out[4]) {
  uint8_t *m = (uint8_t *)malloc(len + 8);
  for (int i = 0; i < 8; i++) m[i] = (uint8_t)((u64)len >> (8 * i));
  if (len) memcpy(m + 8, state, len);
  u64 h = orc_siphash(m, len + 8, 0, 0, 1, 3);
  free(m);
  uint8_t seed[32];
  for (int k = 0; k < 4; k++)
    for (int i = 0; i < 8; i++) seed[8 * k + i] = (uint8_t)(h >> (8 * i));
  rng_t g;
  rng_init(&g, seed);
  fr_rand(&g, out);
}
static void tr_challenge(tr_t *t, const char *label, u64 out[4]) {
  tr_label(t, label);
  challenge_from_state(t->buf, t->len, out);
}
void orc_transcript_challenge(const uint8_t *state, size_t len, uint64_t out[4]) {
  challenge_from_state(state, len, out);
}

/* ----------------------------------------------------------------- G1 (Jacobian) */
typedef struct { u64 x[4], y[4], z[4]; } jac;

static void jac_zero(jac *p) {
  memcpy(p->x, FQ.one, 32);
  memcpy(p->y, FQ.one, 32);
  memset(p->z, 0, 32);
}
static void jac_dbl(jac *r, const jac *p) {
  if (is_zero4(p->z) || is_zero4(p->y)) { jac_zero(r); return; }
  u64 A[4], B[4], C[4], D[4], E[4], F_[4], t[4], X3[4], Y3[4], Z3[4];
  fmul(&FQ, A, p->x, p->x);
  fmul(&FQ, B, p->y, p->y);
  fmul(&FQ, C, B, B);
  fadd(&FQ, t, p->x, B);
  fmul(&FQ, t, t, t);
  fsub(&FQ, t, t, A);
  fsub(&FQ, t, t, C);
  fadd(&FQ, D, t, t);
  fadd(&FQ, E, A, A);
  fadd(&FQ, E, E, A);
  fmul(&FQ, F_, E, E);
  fsub(&FQ, X3, F_, D);
  fsub(&FQ, X3, X3, D);
  fsub(&FQ, t, D, X3);
  fmul(&FQ, Y3, E, t);
  fadd(&FQ, t, C, C);
  fadd(&FQ, t, t, t);
  fadd(&FQ, t, t, t);
  fsub(&FQ, Y3, Y3, t);
  fmul(&FQ, Z3, p->y, p->z);
  fadd(&FQ, Z3, Z3, Z3);
  memcpy(r->x, X3, 32);
  memcpy(r->y, Y3, 32);
  memcpy(r->z, Z3, 32);
}
static void jac_add(jac *r, const jac *p, const jac *q) {
  if (is_zero4(p->z)) { *r = *q; return; }
  if (is_zero4(q->z)) { *r = *p; return; }
  u64 Z1Z1[4], Z2Z2[4], U1[4], U2[4], S1[4], S2[4], H[4], I[4], J[4], rr[4], V[4], t[4];
  jac o;
  fmul(&FQ, Z1Z1, p->z, p->z);
  fmul(&FQ, Z2Z2, q->z, q->z);
  fmul(&FQ, U1, p->x, Z2Z2);
  fmul(&FQ, U2, q->x, Z1Z1);
  fmul(&FQ, S1, p->y, q->z);
  fmul(&FQ, S1, S1, Z2Z2);
  fmul(&FQ, S2, q->y, p->z);
  fmul(&FQ, S2, S2, Z1Z1);
  if (eq4(U1, U2)) {
    if (eq4(S1, S2)) { jac_dbl(r, p); return; }
    jac_zero(r);
    return;
  }
  fsub(&FQ, H, U2, U1);
  fadd(&FQ, I, H, H);
  fmul(&FQ, I, I, I);
  fmul(&FQ, J, H, I);
  fsub(&FQ, rr, S2, S1);
  fadd(&FQ, rr, rr, rr);
  fmul(&FQ, V, U1, I);
  fmul(&FQ, o.x, rr, rr);
  fsub(&FQ, o.x, o.x, J);
  fsub(&FQ, o.x, o.x, V);
  fsub(&FQ, o.x, o.x, V);
  fsub(&FQ, t, V, o.x);
  fmul(&FQ, o.y, rr, t);
  fmul(&FQ, t, S1, J);
  fadd(&FQ, t, t, t);
  fsub(&FQ, o.y, o.y, t);
  fadd(&FQ, t, p->z, q->z);
  fmul(&FQ, t, t, t);
  fsub(&FQ, t, t, Z1Z1);
  fsub(&FQ, t, t, Z2Z2);
  fmul(&FQ, o.z, t, H);
  *r = o;
}
static void aff_to_jac(jac *r, const u64 a[8]) {
  if (is_zero4(a) && is_zero4(a + 4)) { jac_zero(r); return; }
  memcpy(r->x, a, 32);
  memcpy(r->y, a + 4, 32);
  memcpy(r->z, FQ.one, 32);
}
static void jac_to_aff(u64 a[8], const jac *p) {
  if (is_zero4(p->z)) { memset(a, 0, 64); return; }
  u64 zi[4], zi2[4], zi3[4];
  finv(&FQ, zi, p->z);
  fmul(&FQ, zi2, zi, zi);
  fmul(&FQ, zi3, zi2, zi);
  fmul(&FQ, a, p->x, zi2);
  fmul(&FQ, a + 4, p->y, zi3);
}
/* G1Projective * Fr: double-and-add over the canonical scalar bits */
static void jac_mul(jac *r, const jac *p, const u64 s_mont[4]) {
  u64 k[4];
  from_mont(&FR, k, s_mont);
  jac acc;
  jac_zero(&acc);
  for (int i = 255; i >= 0; i--) {
    jac_dbl(&acc, &acc);
    if ((k[i / 64] >> (i % 64)) & 1) jac_add(&acc, &acc, p);
  }
  *r = acc;
}

/* ----------------------------------------------------------------- setup_params */
static size_t next_pow2(size_t n) {
  size_t p = 1;
  while (p < n) p <<= 1;
  return p;
}
size_t orc_setup_num_powers(unsigned log_size) {
  size_t max_ops = (size_t)1 << (log_size + 2);
  return next_pow2(max_ops) + 1;
}
void orc_setup_params(unsigned log_size, uint64_t tau_out[4], uint8_t seed_out[32],
                      uint64_t *g1_powers_out) {
  uint8_t s42[32];
  memset(s42, 42, 32);
  rng_t g;
  rng_init(&g, s42);
  u64 tau[4];
  fr_rand(&g, tau); /* src/utils.rs:84 */
  memcpy(tau_out, tau, 32);
  if (g1_powers_out) { /* src/utils.rs:89-96 */
    size_t n = orc_setup_num_powers(log_size);
    jac gen;
    u64 gaff[8] = {0};
    u64 one_c[4] = {1, 0, 0, 0}, two_c[4] = {2, 0, 0, 0};
    to_mont(&FQ, gaff, one_c);
    to_mont(&FQ, gaff + 4, two_c);
    aff_to_jac(&gen, gaff);
    u64 cur[4];
    memcpy(cur, FR.one, 32);
    for (size_t i = 0; i < n; i++) {
      jac P;
      jac_mul(&P, &gen, cur);
      jac_to_aff(g1_powers_out + 8 * i, &P);
      fmul(&FR, cur, cur, tau);
    }
  }
  /* src/utils.rs:101-102: fill_bytes consumes whole u32 words */
  for (int w = 0; w < 8; w++) {
    uint32_t v = rng_u32(&g);
    for (int i = 0; i < 4; i++) seed_out[4 * w + i] = (uint8_t)(v >> (8 * i));
  }
}

/* ---------------------------------------------------------- lagrange_interpolate */
/* src/polynomials.rs:301-352, verbatim O(n^3) over points (x_i = i, y_i) */
static void lagrange_points(const u64 *xs, const u64 *ys, size_t n, u64 *res) {
  memset(res, 0, n * 32);
  if (!n) return;
  u64 *li = (u64 *)malloc((n + 1) * 32), *nw = (u64 *)malloc((n + 1) * 32);
  for (size_t i = 0; i < n; i++) {
    size_t len = 1;
    memcpy(li, FR.one, 32);
    for (size_t j = 0; j < n; j++) {
      if (i == j) continue;
      u64 den[4], dinv[4], t[4];
      fsub(&FR, den, xs + 4 * i, xs + 4 * j);
      finv(&FR, dinv, den);
      memset(nw, 0, (len + 1) * 32);
      for (size_t k = 0; k < len; k++) fadd(&FR, nw + 4 * (k + 1), nw + 4 * (k + 1), li + 4 * k);
      for (size_t k = 0; k < len; k++) {
        fmul(&FR, t, li + 4 * k, xs + 4 * j);
        fsub(&FR, nw + 4 * k, nw + 4 * k, t);
      }
      for (size_t k = 0; k < len + 1; k++) fmul(&FR, nw + 4 * k, nw + 4 * k, dinv);
      len++;
      u64 *sw = li; li = nw; nw = sw;
    }
    for (size_t k = 0; k < len && k < n; k++) {
      u64 t[4];
      fmul(&FR, t, ys + 4 * i, li + 4 * k);
      fadd(&FR, res + 4 * k, res + 4 * k, t);
    }
  }
  free(li);
  free(nw);
}
void orc_interpolate_consecutive(const uint64_t *y, size_t n, uint64_t *coeffs) {
  u64 *xs = (u64 *)malloc((n ? n : 1) * 32);
  for (size_t i = 0; i < n; i++) fr_u64(xs + 4 * i, i);
  lagrange_points(xs, y, n, coeffs);
  free(xs);
}

/* ----------------------------------------------------------------- KZG */
int orc_commit(const uint64_t *g1, size_t n_powers, const uint64_t *c, size_t n,
               uint64_t out[8]) {
  if (n > n_powers) return 4; /* src/commitments.rs:166-170 */
  jac acc;
  jac_zero(&acc);
  for (size_t i = 0; i < n; i++) { /* src/commitments.rs:173-177 */
    jac P, T;
    aff_to_jac(&P, g1 + 8 * i);
    jac_mul(&T, &P, c + 4 * i);
    jac_add(&acc, &acc, &T);
  }
  jac_to_aff(out, &acc);
  return 0;
}
static void horner(const u64 *c, size_t n, const u64 z[4], u64 out[4]) {
  u64 acc[4] = {0, 0, 0, 0};
  for (size_t i = n; i-- > 0;) {
    fmul(&FR, acc, acc, z);
    fadd(&FR, acc, acc, c + 4 * i);
  }
  memcpy(out, acc, 32);
}
int orc_open(const uint64_t *g1, size_t n_powers, const uint64_t *c, size_t n,
             const uint64_t z[4], uint64_t value[4], uint64_t proof[8]) {
  horner(c, n, z, value); /* src/commitments.rs:305-313 */
  if (n < 2) { /* polynomial_division: remainder shorter than divisor -> empty quotient */
    memset(proof, 0, 64);
    return 0;
  }
  /* src/commitments.rs:317-375: long division of (P - v) by (x - z); leading coeff 1 */
  u64 *rem = (u64 *)malloc(n * 32), *q = (u64 *)malloc((n - 1) * 32);
  memcpy(rem, c, n * 32);
  fsub(&FR, rem, rem, value);
  u64 mz[4];
  fneg(&FR, mz, z);
  for (size_t i = n - 1; i-- > 0;) {
    u64 co[4], t[4];
    memcpy(co, rem + 4 * (i + 1), 32);
    memcpy(q + 4 * i, co, 32);
    fmul(&FR, t, co, mz);
    fsub(&FR, rem + 4 * i, rem + 4 * i, t);
    memset(rem + 4 * (i + 1), 0, 32);
  }
  int st = orc_commit(g1, n_powers, q, n - 1, proof);
  free(rem);
  free(q);
  return st;
}
void orc_commitment_hash(const uint64_t aff[8], uint64_t out[4]) {
  /* src/commitments.rs:73-84: canonical affine x as LE bytes, reduced mod r */
  u64 x[4];
  from_mont(&FQ, x, aff);
  while (geq(x, FR.m)) sub4(x, x, FR.m);
  to_mont(&FR, out, x);
}

/* ----------------------------------------------------------------- MLE */
static void mle_eval(const u64 *ev, unsigned nv, const u64 *pt, u64 out[4]) {
  /* src/polynomials.rs:85-122 (sum order irrelevant: exact arithmetic) */
  u64 acc[4] = {0, 0, 0, 0};
  u64 *omr = (u64 *)malloc((nv ? nv : 1) * 32);
  for (unsigned j = 0; j < nv; j++) fsub(&FR, omr + 4 * j, FR.one, pt + 4 * j);
  size_t N = (size_t)1 << nv;
  for (size_t i = 0; i < N; i++) {
    if (is_zero4(ev + 4 * i)) continue;
    u64 b[4];
    memcpy(b, FR.one, 32);
    for (unsigned j = 0; j < nv; j++) fmul(&FR, b, b, ((i >> j) & 1) ? pt + 4 * j : omr + 4 * j);
    fmul(&FR, b, b, ev + 4 * i);
    fadd(&FR, acc, acc, b);
  }
  free(omr);
  memcpy(out, acc, 32);
}
void orc_mle_evaluate(const uint64_t *ev, unsigned nv, const uint64_t *pt, uint64_t out[4]) {
  mle_eval(ev, nv, pt, out);
}
void orc_mle_partial_evaluate(const uint64_t *ev, unsigned nv, const uint64_t *fixed, unsigned k,
                              uint64_t *out) {
  if (k == 0) { memcpy(out, ev, ((size_t)32) << nv); return; }
  unsigned nn = nv - k;
  u64 *pt = (u64 *)malloc((size_t)nv * 32);
  memcpy(pt, fixed, (size_t)k * 32);
  for (size_t idx = 0; idx < ((size_t)1 << nn); idx++) {
    for (unsigned j = 0; j < nn; j++) {
      if ((idx >> j) & 1) memcpy(pt + 4 * (k + j), FR.one, 32);
      else memset(pt + 4 * (k + j), 0, 32);
    }
    mle_eval(ev, nv, pt, out + 4 * idx);
  }
  free(pt);
}

/* ----------------------------------------------------------------- SumCheck */
typedef struct {
  const u64 *const *tables;
  int n_tables;
  unsigned nv;
  int n_terms;
  const u64 *coeffs;
  const int *tt;
  int *used; /* which tables the closure evaluates */
} closure_t;

static void closure_eval(const closure_t *C, const u64 *pt, u64 out[4]) {
  /* the reference closures evaluate every captured MLE at the point (src/twist.rs:197-199) */
  u64 vals[16][4];
  for (int t = 0; t < C->n_tables && t < 16; t++)
    if (C->used[t]) mle_eval(C->tables[t], C->nv, pt, vals[t]);
  u64 acc[4] = {0, 0, 0, 0};
  for (int t = 0; t < C->n_terms; t++) {
    u64 p[4];
    memcpy(p, C->coeffs + 4 * t, 32);
    for (int j = 0; j < 3; j++) {
      int ix = C->tt[3 * t + j];
      if (ix >= 0) fmul(&FR, p, p, vals[ix]);
    }
    fadd(&FR, acc, acc, p);
  }
  memcpy(out, acc, 32);
}

static int sumcheck_core(const closure_t *C, unsigned nv, const u64 claimed[4], tr_t *tr,
                         u64 *rounds_out, u64 final_out[4], u64 *chal_out) {
  u64 cur[4];
  memcpy(cur, claimed, 32);
  u64 *pt = (u64 *)malloc((nv ? nv : 1) * 32);
  u64 xs[4][4], ev[4][4], coeffs[4][4];
  for (int i = 0; i < 4; i++) fr_u64(xs[i], (u64)i);
  for (unsigned rnd = 0; rnd < nv; rnd++) {
    unsigned rem = nv - rnd - 1;
    for (int xv = 0; xv < 4; xv++) { /* src/sumcheck.rs:175-198 */
      u64 s[4] = {0, 0, 0, 0};
      for (size_t suf = 0; suf < ((size_t)1 << rem); suf++) {
        memcpy(pt + 4 * rnd, xs[xv], 32);
        for (unsigned b = 0; b < rem; b++) {
          if ((suf >> b) & 1) memcpy(pt + 4 * (rnd + 1 + b), FR.one, 32);
          else memset(pt + 4 * (rnd + 1 + b), 0, 32);
        }
        u64 f[4];
        closure_eval(C, pt, f);
        fadd(&FR, s, s, f);
      }
      memcpy(ev[xv], s, 32);
    }
    lagrange_points(&xs[0][0], &ev[0][0], 4, &coeffs[0][0]); /* :201-206 */
    u64 g0[4], g1[4], sum[4];
    horner(&coeffs[0][0], 4, xs[0], g0);
    horner(&coeffs[0][0], 4, xs[1], g1);
    fadd(&FR, sum, g0, g1);
    if (!eq4(sum, cur)) { free(pt); return 6; } /* :80-84 */
    memcpy(rounds_out + 16 * rnd, coeffs, 128);
    char lab[64];
    snprintf(lab, sizeof lab, "sumcheck_round_%u", rnd);
    tr_label(tr, lab);
    for (int i = 0; i < 4; i++) tr_fr(tr, coeffs[i]);
    snprintf(lab, sizeof lab, "sumcheck_challenge_%u", rnd);
    u64 ch[4];
    tr_challenge(tr, lab, ch);
    memcpy(pt + 4 * rnd, ch, 32);
    if (chal_out) memcpy(chal_out + 4 * rnd, ch, 32);
    horner(&coeffs[0][0], 4, ch, cur);
  }
  closure_eval(C, pt, final_out); /* :104 */
  free(pt);
  return 0;
}

int orc_sumcheck_prove(const uint64_t *const *tables, int n_tables, unsigned nv,
                       const uint64_t *claimed_sum, int n_terms, const uint64_t *term_coeffs,
                       const int *term_tables, const uint8_t *prefix, size_t prefix_len,
                       uint64_t *rounds_out, uint64_t final_out[4], uint64_t *challenges_out) {
  int used[16] = {0};
  for (int t = 0; t < n_terms; t++)
    for (int j = 0; j < 3; j++)
      if (term_tables[3 * t + j] >= 0) used[term_tables[3 * t + j]] = 1;
  closure_t C = {tables, n_tables, nv, n_terms, term_coeffs, term_tables, used};
  tr_t tr;
  tr_init(&tr);
  if (prefix_len) tr_put(&tr, prefix, prefix_len);
  int st = sumcheck_core(&C, nv, claimed_sum, &tr, rounds_out, final_out, challenges_out);
  tr_free(&tr);
  return st;
}

/* ----------------------------------------------------------------- Twist / Shout */
static unsigned log2_exact(size_t n) {
  unsigned l = 0;
  while (((size_t)1 << l) < n) l++;
  return l;
}

static int prove_common(const uint64_t *g1, size_t n_powers, const u64 *vecA, size_t nA,
                        const u64 *vecB, size_t nB, const char *labA, const char *labB,
                        const u64 *const *mles, int n_mles, unsigned nv, orc_proof *out) {
  memset(out, 0, sizeof *out);
  u64 *pa = (u64 *)malloc((nA ? nA : 1) * 32), *pb = (u64 *)malloc((nB ? nB : 1) * 32);
  orc_interpolate_consecutive(vecA, nA, pa); /* vector_to_polynomial x2 */
  orc_interpolate_consecutive(vecB, nB, pb);
  int st = orc_commit(g1, n_powers, pa, nA, out->commitment[0]);
  if (!st) st = orc_commit(g1, n_powers, pb, nB, out->commitment[1]);
  if (st) { free(pa); free(pb); return st; }
  tr_t tr;
  tr_init(&tr);
  u64 h[4];
  orc_commitment_hash(out->commitment[0], h);
  tr_label(&tr, labA);
  tr_fr(&tr, h);
  orc_commitment_hash(out->commitment[1], h);
  tr_label(&tr, labB);
  tr_fr(&tr, h);
  /* constraint closure: evaluates every MLE, returns zero (src/twist.rs:191-213) */
  int used[16] = {0};
  for (int i = 0; i < n_mles; i++) used[i] = 1;
  closure_t C = {mles, n_mles, nv, 0, NULL, NULL, used};
  u64 zero[4] = {0, 0, 0, 0};
  out->num_rounds = nv;
  st = sumcheck_core(&C, nv, zero, &tr, &out->round_polynomials[0][0][0], out->final_evaluation,
                     &out->sumcheck_challenges[0][0]);
  if (!st && nv > 0) {
    /* challenge_field_elements("opening_challenges", nv); only _0 is used */
    u64 z[4];
    tr_challenge(&tr, "opening_challenges_0", z);
    memcpy(out->opening_point, z, 32);
    for (unsigned i = 1; i < nv; i++) {
      char lab[64];
      u64 dummy[4];
      snprintf(lab, sizeof lab, "opening_challenges_%u", i);
      tr_challenge(&tr, lab, dummy);
    }
    st = orc_open(g1, n_powers, pa, nA, z, out->final_evaluations[0], out->opening_proofs[0]);
    if (!st) st = orc_open(g1, n_powers, pb, nB, z, out->final_evaluations[1], out->opening_proofs[1]);
    out->num_openings = 2;
  }
  tr_free(&tr);
  free(pa);
  free(pb);
  return st;
}

int orc_twist_prove(const uint64_t *g1, size_t n_powers, size_t max_ops, const uint64_t *addr,
                    const uint64_t *val, const uint8_t *is_write, size_t n_ops, orc_proof *out) {
  if (n_ops > max_ops) return 1; /* src/twist.rs:108-112 */
  size_t N = next_pow2(n_ops); /* :141 (next_power_of_two().max(1)) */
  u64 *A = (u64 *)calloc(N, 32), *V = (u64 *)calloc(N, 32), *O = (u64 *)calloc(N, 32);
  for (size_t i = 0; i < n_ops; i++) {
    memcpy(A + 4 * i, addr + 4 * i, 32);
    memcpy(V + 4 * i, val + 4 * i, 32);
    if (is_write[i]) memcpy(O + 4 * i, FR.one, 32);
  }
  const u64 *mles[3] = {A, V, O};
  int st = prove_common(g1, n_powers, A, N, V, N, "address_commitment", "value_commitment", mles, 3,
                        log2_exact(N), out);
  free(A); free(V); free(O);
  return st;
}

int orc_shout_prove(const uint64_t *g1, size_t n_powers, size_t max_ops, const uint64_t *entries,
                    size_t n_entries, const uint64_t *indices, size_t n_lookups, orc_proof *out) {
  if (n_lookups > max_ops) return 1; /* src/shout.rs:98-102 */
  size_t T = next_pow2(n_entries), M = next_pow2(n_lookups);
  u64 *Tb = (u64 *)calloc(T, 32), *I = (u64 *)calloc(M, 32);
  memcpy(Tb, entries, n_entries * 32);
  memcpy(I, indices, n_lookups * 32);
  const u64 *mles[1] = {I};
  int st = prove_common(g1, n_powers, Tb, T, I, M, "table_commitment", "index_commitment", mles, 1,
                        log2_exact(M), out);
  free(Tb); free(I);
  return st;
}

/* Horner evaluation (src/utils.rs:217-221), exposed for size-independent checks. */
void orc_horner(const uint64_t *c, size_t n, const uint64_t z[4], uint64_t out[4]) { horner(c, n, z, out); }
