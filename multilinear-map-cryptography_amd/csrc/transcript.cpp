// transcript.cpp -- host-side Fiat-Shamir transcript and RNG of the prover.
//
// Restates src/utils.rs:134-204 (Transcript) and the third-party pieces it relies on:
//   * rand_chacha 0.3.1 ChaCha20Rng::from_seed -- DJB ChaCha20 (20 rounds), key = seed,
//     64-bit block counter from 0, stream id 0, output read as LE u32 words;
//   * ark-ff 0.4.2 UniformRand for Fr -- 4 x next_u64 (lo word first), clear the top
//     two bits, reject >= r, and keep the limbs AS the Montgomery representation;
//   * Rust std DefaultHasher (SipHash-1-3, keys 0/0) over Vec<u8>: write_usize(len)
//     then the raw bytes.
// The sequential transcript sits between device kernels (one challenge per
// sum-check round); it is a few KB and costs microseconds.
#include <cstring>

#include "common.hpp"

namespace tns {

static inline uint32_t rotl32(uint32_t v, int c) { return (v << c) | (v >> (32 - c)); }
static inline uint64_t rotl64(uint64_t v, int c) { return (v << c) | (v >> (64 - c)); }

void chacha20_block_host(const uint32_t key[8], uint64_t counter, uint32_t out[16]) {
  uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};
  std::memcpy(s + 4, key, 32);
  s[12] = (uint32_t)counter;
  s[13] = (uint32_t)(counter >> 32);
  s[14] = s[15] = 0;
  uint32_t x[16];
  std::memcpy(x, s, sizeof s);
  auto q = [&](int a, int b, int c, int d) {
    x[a] += x[b]; x[d] = rotl32(x[d] ^ x[a], 16);
    x[c] += x[d]; x[b] = rotl32(x[b] ^ x[c], 12);
    x[a] += x[b]; x[d] = rotl32(x[d] ^ x[a], 8);
    x[c] += x[d]; x[b] = rotl32(x[b] ^ x[c], 7);
  };
  for (int r = 0; r < 10; r++) {
    q(0, 4, 8, 12); q(1, 5, 9, 13); q(2, 6, 10, 14); q(3, 7, 11, 15);
    q(0, 5, 10, 15); q(1, 6, 11, 12); q(2, 7, 8, 13); q(3, 4, 9, 14);
  }
  for (int i = 0; i < 16; i++) out[i] = x[i] + s[i];
}

namespace {
// rand_core BlockRng over ChaCha20 (a 4-block buffer there: the word stream is blocks 0, 1, 2, ...
// in order either way, so blocks are made one at a time here -- a challenge's Fr::rand reads 8
// words, and the other three blocks were 0.6 us of every sum-check round's host turn)
struct ChaChaStream {
  uint32_t key[8];
  uint64_t ctr = 0;
  uint32_t buf[16];
  int pos = 16;
  explicit ChaChaStream(const uint8_t seed[32]) {
    for (int i = 0; i < 8; i++)
      key[i] = (uint32_t)seed[4 * i] | (uint32_t)seed[4 * i + 1] << 8 |
               (uint32_t)seed[4 * i + 2] << 16 | (uint32_t)seed[4 * i + 3] << 24;
  }
  uint32_t word() {
    if (pos == 16) {
      chacha20_block_host(key, ctr++, buf);
      pos = 0;
    }
    return buf[pos++];
  }
  uint64_t u64() {
    uint64_t lo = word();
    return lo | (uint64_t)word() << 32;
  }
};

Fr fr_rand(ChaChaStream &g) {
  for (;;) {
    uint64_t l[4];
    for (int i = 0; i < 4; i++) l[i] = g.u64();
    l[3] &= ~0ULL >> 2;
    Fr r;
    for (int i = 0; i < 4; i++) {
      r.v[2 * i] = (uint32_t)l[i];
      r.v[2 * i + 1] = (uint32_t)(l[i] >> 32);
    }
    // accept iff limbs < r (compare as a 256-bit integer)
    bool less = false, decided = false;
    for (int i = 7; i >= 0 && !decided; i--) {
      if (r.v[i] != FrCfg::M[i]) {
        less = r.v[i] < FrCfg::M[i];
        decided = true;
      }
    }
    if (decided && less) return r;
  }
}
}  // namespace

Fr host_fr_rand_chacha(const uint8_t seed[32], uint8_t *fs_seed_out) {
  ChaChaStream g(seed);
  Fr r = fr_rand(g);
  if (fs_seed_out) {  // RngCore::fill_bytes takes whole u32 words
    for (int w = 0; w < 8; w++) {
      uint32_t v = g.word();
      for (int i = 0; i < 4; i++) fs_seed_out[4 * w + i] = (uint8_t)(v >> (8 * i));
    }
  }
  return r;
}

void host_fr_rand_stream(const uint8_t seed[32], size_t n, Fr *out) {
  ChaChaStream g(seed);
  for (size_t i = 0; i < n; i++) out[i] = fr_rand(g);
}

// SipHash-1-3 with zero keys (Rust's DefaultHasher) over  prefix (8 bytes, if has_prefix) || m[0..n):
// Hash for [u8] writes the length first, and the message is hashed in place (no concatenated copy).
// resume (optional): the state after the prefix and m's first `skip` bytes (skip % 8 == 0), from
// HostTranscript::prehash -- only m[skip, n) is absorbed here.
static uint64_t siphash13_keys00_pre(bool has_prefix, uint64_t prefix, const uint8_t *m, size_t n,
                                     const uint64_t *resume = nullptr, size_t skip = 0, uint64_t *save = nullptr) {
  uint64_t v0 = 0x736f6d6570736575ULL, v1 = 0x646f72616e646f6dULL;
  uint64_t v2 = 0x6c7967656e657261ULL, v3 = 0x7465646279746573ULL;
  auto round = [&]() {
    v0 += v1; v1 = rotl64(v1, 13); v1 ^= v0; v0 = rotl64(v0, 32);
    v2 += v3; v3 = rotl64(v3, 16); v3 ^= v2;
    v0 += v3; v3 = rotl64(v3, 21); v3 ^= v0;
    v2 += v1; v1 = rotl64(v1, 17); v1 ^= v2; v2 = rotl64(v2, 32);
  };
  auto block = [&](uint64_t w) {
    v3 ^= w;
    round();
    v0 ^= w;
  };
  size_t i = 0;
  if (resume) {
    v0 = resume[0];
    v1 = resume[1];
    v2 = resume[2];
    v3 = resume[3];
    i = skip;
  } else if (has_prefix) {
    block(prefix);  // (8 bytes: a whole block, the message stays block-aligned)
  }
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    std::memcpy(&w, m + i, 8);  // little-endian host
    block(w);
  }
  if (save) {  // (prehash: the whole blocks only, no finalisation)
    save[0] = v0;
    save[1] = v1;
    save[2] = v2;
    save[3] = v3;
    return 0;
  }
  const size_t total = n + (has_prefix ? 8 : 0);
  uint64_t b = (uint64_t)(total & 0xff) << 56;
  for (size_t j = 0; i + j < n; j++) b |= (uint64_t)m[i + j] << (8 * j);
  block(b);
  v2 ^= 0xff;
  round();
  round();
  round();
  return v0 ^ v1 ^ v2 ^ v3;
}

uint64_t siphash13_keys00(const uint8_t *m, size_t n) { return siphash13_keys00_pre(false, 0, m, n); }

void HostTranscript::append_label(const char *s) { append_bytes((const uint8_t *)s, std::strlen(s)); }
void HostTranscript::append_bytes(const uint8_t *p, size_t n) { state.insert(state.end(), p, p + n); }
void HostTranscript::append_fr(const Fr &x) {
  Fr c = from_mont(x);  // compressed serialisation: 32-byte LE canonical
  uint8_t b[32];
  for (int i = 0; i < 8; i++)
    for (int k = 0; k < 4; k++) b[4 * i + k] = (uint8_t)(c.v[i] >> (8 * k));
  append_bytes(b, 32);
}
void HostTranscript::prehash(size_t final_len) {
  pre.valid = false;
  if (final_len < state.size()) return;
  const size_t whole = state.size() / 8 * 8;
  siphash13_keys00_pre(true, (uint64_t)final_len, state.data(), whole, nullptr, 0, pre.v);
  pre.final_len = final_len;
  pre.done = whole;
  pre.valid = true;
}
Fr HostTranscript::challenge_bytes(const uint8_t *label, size_t n) {
  append_bytes(label, n);
  // Hash for [u8]: write_usize(len) first, then the bytes (resumed after the prehashed blocks when
  // the state reached the length prehash assumed)
  const bool resume = pre.valid && pre.final_len == state.size() && pre.done <= state.size();
  const uint64_t h = siphash13_keys00_pre(true, (uint64_t)state.size(), state.data(), state.size(),
                                          resume ? pre.v : nullptr, resume ? pre.done : 0);
  pre.valid = false;
  uint8_t seed[32];
  for (int k = 0; k < 4; k++) std::memcpy(seed + 8 * k, &h, 8);  // hash.to_le_bytes() x 4
  ChaChaStream g(seed);
  return fr_rand(g);
}
Fr HostTranscript::challenge(const char *label) {
  return challenge_bytes((const uint8_t *)label, std::strlen(label));
}

// KZGCommitmentValue::hash (src/commitments.rs:73-84): affine x, canonical LE bytes,
// reduced modulo r.  The identity's affine x is 0.
Fr commitment_hash(const G1Affine &a) {
  if (a.is_inf()) return Fr::zero();
  Fq xc = from_mont(a.x);
  Fr t;
  for (int i = 0; i < 8; i++) t.v[i] = xc.v[i];
  // x < p < 2r: at most one subtraction of r
  reduce_once(t);
  return to_mont(t);
}

Fr horner_host(const Fr *c, int n, const Fr &z) {
  Fr acc = Fr::zero();
  for (int i = n - 1; i >= 0; i--) acc = add(mul(acc, z), c[i]);
  return acc;
}

// Unique cubic through (0,e0),(1,e1),(2,e2),(3,e3) -- the value lagrange_interpolate
// returns for the 4 round points (src/sumcheck.rs:201-206).
void interpolate4_host(const Fr e[4], Fr out[4]) {
  // Newton forward differences then expand x(x-1)(x-2).
  Fr d1 = sub(e[1], e[0]), d1b = sub(e[2], e[1]), d1c = sub(e[3], e[2]);
  Fr d2 = sub(d1b, d1), d2b = sub(d1c, d1b);
  Fr d3 = sub(d2b, d2);
  // (the two constants once: two Fermat inversions per round were ~20 us of every sum-check
  // round's host turn)
  static const Fr inv2 = inv(from_u64<FrCfg>(2)), inv6 = inv(from_u64<FrCfg>(6));
  Fr a0 = e[0], a1 = d1, a2 = mul(d2, inv2), a3 = mul(d3, inv6);
  // f = a0 + a1 x + a2 x(x-1) + a3 x(x-1)(x-2)
  //   = a0 + (a1 - a2 + 2 a3) x + (a2 - 3 a3) x^2 + a3 x^3
  out[0] = a0;
  out[1] = add(sub(a1, a2), dbl(a3));
  out[2] = sub(a2, mul3(a3));
  out[3] = a3;
}

}  // namespace tns
