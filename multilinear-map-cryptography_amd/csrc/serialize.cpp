// serialize.cpp -- the proof wire format, host side.
//
// KZGCommitmentValue / KZGProof serialize as their G1 point (src/commitments.rs:94-154), i.e.
// ark-ec 0.4.2 short-Weierstrass Affine::serialize_with_mode / ark-serialize 0.4.2:
//   compressed:   x as 32 bytes little-endian (canonical), flags in the top two bits of the
//                 last byte: 0x80 = YIsNegative (y > -y as integers), 0x40 = PointAtInfinity
//                 (x = y = 0 then);
//   uncompressed: x (32 bytes LE) then y (32 bytes LE) carrying the same flags.
// Fr: 32 bytes LE canonical.  Proof structs: their fields in declaration order
// (src/twist.rs:76-89, src/shout.rs:64-79, src/sumcheck.rs:25-31), Vec<T> as a u64 LE length
// followed by the elements -- the layout #[derive(CanonicalSerialize)] produces.
#include <cstring>
#include <string>
#include <vector>

#include "common.hpp"

namespace tns {

namespace {

constexpr uint8_t FLAG_NEG = 0x80, FLAG_INF = 0x40;

void put_le(const Fp<FqCfg> &canon, uint8_t *out) {
  for (int i = 0; i < 8; i++)
    for (int b = 0; b < 4; b++) out[4 * i + b] = (uint8_t)(canon.v[i] >> (8 * b));
}
template <class C>
Fp<C> get_le(const uint8_t *in) {
  Fp<C> r;
  for (int i = 0; i < 8; i++) {
    uint32_t w = 0;
    for (int b = 0; b < 4; b++) w |= (uint32_t)in[4 * i + b] << (8 * b);
    r.v[i] = w;
  }
  return r;
}
template <class C>
bool lt_modulus(const Fp<C> &x) {
  for (int i = 7; i >= 0; i--) {
    if (x.v[i] < C::M[i]) return true;
    if (x.v[i] > C::M[i]) return false;
  }
  return false;
}
template <class C>
bool gt_raw(const Fp<C> &a, const Fp<C> &b) {
  for (int i = 7; i >= 0; i--) {
    if (a.v[i] != b.v[i]) return a.v[i] > b.v[i];
  }
  return false;
}
// y is "negative" when y > -y as canonical integers (ark-ec to_flags: y <= -y is positive)
bool y_negative(const Fq &y_mont) {
  const Fq y = from_mont(y_mont), ny = from_mont(neg(y_mont));
  return gt_raw(y, ny);
}
// square root in Fq (p = 3 mod 4): a^((p+1)/4); false if a is not a square
bool fq_sqrt(const Fq &a, Fq *out) {
  u32 e[8];
  // (p + 1) / 4
  uint64_t carry = 1;
  u32 t[8];
  for (int i = 0; i < 8; i++) {
    uint64_t s = (uint64_t)FqCfg::M[i] + carry;
    t[i] = (u32)s;
    carry = s >> 32;
  }
  for (int i = 0; i < 8; i++) e[i] = (t[i] >> 2) | (i < 7 ? (t[i + 1] << 30) : 0);
  const Fq r = pow_limbs(a, e);
  *out = r;
  return sqr(r) == a;
}

}  // namespace

void g1_serialize(const G1Affine &P, bool compressed, uint8_t *out) {
  const size_t n = compressed ? 32 : 64;
  std::memset(out, 0, n);
  uint8_t flags;
  if (P.is_inf()) {
    flags = FLAG_INF;
  } else {
    put_le(from_mont(P.x), out);
    if (!compressed) put_le(from_mont(P.y), out + 32);
    flags = y_negative(P.y) ? FLAG_NEG : 0;
  }
  out[n - 1] |= flags;
}

G1Affine g1_deserialize(const uint8_t *in, bool compressed, bool validate) {
  const size_t n = compressed ? 32 : 64;
  uint8_t buf[64];
  std::memcpy(buf, in, n);
  const uint8_t flags = buf[n - 1] & (FLAG_NEG | FLAG_INF);
  buf[n - 1] &= (uint8_t)~(FLAG_NEG | FLAG_INF);
  if (flags == (FLAG_NEG | FLAG_INF)) throw Error(TNS_ERR_INVALID_PARAMETERS, "invalid G1 flags");
  G1Affine P;
  P.x = Fq::zero();
  P.y = Fq::zero();
  if (flags & FLAG_INF) return P;  // identity (x = y = 0)
  const Fq xc = get_le<FqCfg>(buf);
  if (!lt_modulus(xc)) throw Error(TNS_ERR_INVALID_PARAMETERS, "G1 x not below the field modulus");
  P.x = to_mont(xc);
  if (compressed) {
    const Fq rhs = add(mul(sqr(P.x), P.x), from_u64<FqCfg>(3));
    Fq y;
    if (!fq_sqrt(rhs, &y)) throw Error(TNS_ERR_INVALID_PARAMETERS, "G1 x is not on the curve");
    if (y_negative(y) != ((flags & FLAG_NEG) != 0)) y = neg(y);
    P.y = y;
  } else {
    const Fq yc = get_le<FqCfg>(buf + 32);
    if (!lt_modulus(yc)) throw Error(TNS_ERR_INVALID_PARAMETERS, "G1 y not below the field modulus");
    P.y = to_mont(yc);
    if (validate && !g1_on_curve(P)) throw Error(TNS_ERR_INVALID_PARAMETERS, "G1 point not on the curve");
  }
  return P;  // BN254 G1 has cofactor 1: on the curve = in the subgroup
}

void fr_serialize(const Fr &x, uint8_t out[32]) {
  const Fr c = from_mont(x);
  for (int i = 0; i < 8; i++)
    for (int b = 0; b < 4; b++) out[4 * i + b] = (uint8_t)(c.v[i] >> (8 * b));
}

Fr fr_deserialize(const uint8_t in[32]) {
  const Fr c = get_le<FrCfg>(in);
  if (!lt_modulus(c)) throw Error(TNS_ERR_INVALID_PARAMETERS, "Fr not below the scalar modulus");
  return to_mont(c);
}

}  // namespace tns
