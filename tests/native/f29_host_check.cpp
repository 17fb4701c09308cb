// f29_host_check.cpp -- the radix-2^29 mixed addition (tools/f29.hpp, the accumulation experiment)
// on the host against the radix-2^32 XYZZ madd of bn254.hpp: 20000 chains of 1..9 additions of
// random, near-M and small coordinates with random signs, compared as affine points.  Built and run
// by tests/test_f29_host.py (g++; the device qualifiers compile away).
#define __device__
#define __forceinline__ inline
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "bn254.hpp"
#include "f29.hpp"
using namespace tns;
static uint64_t s = 88172645463325252ULL;
static u32 rnd() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (u32)s; }
static Fq rand_canon(int kind) {  // kind 0 random < M, 1 near M, 2 small
  Fq r;
  for (int i = 0; i < 8; i++) r.v[i] = rnd();
  if (kind == 1) { for (int i = 0; i < 8; i++) r.v[i] = FqCfg::M[i]; u32 d = rnd() & 0xffff; r.v[0] -= d + 1; }
  else if (kind == 2) { for (int i = 2; i < 8; i++) r.v[i] = 0; }
  else { r.v[7] &= 0x3fffffff; reduce_once(r); reduce_once(r); }
  return r;
}
int main() {
  int bad = 0;
  // algebraic check: run the same chains where the reference takes q as (value * 2^-5) so both see one point
  s = 12345;
  const Fq ic = inv(from_u64<FqCfg>(32));
  for (int chain = 0; chain < 20000; chain++) {
    const int len = 1 + chain % 9;
    G1Xyzz ref = G1Xyzz::inf();
    G1Xyzz29 p; bool empty = true;
    for (int k = 0; k < len; k++) {
      Fq x = rand_canon(rnd() % 3), y = rand_canon(rnd() % 3);  // R' canonical limbs
      bool ng = rnd() & 1;
      G1Affine qr; qr.x = mul(x, ic); qr.y = mul(y, ic); if (ng) qr.y = tns::neg(qr.y);
      ref = xyzz_madd(ref, qr);
      xyzz_madd29(p, empty, f29_from32(x), f29_from32(y), ng);
    }
    G1Xyzz r = G1Xyzz::inf();
    if (!empty) { r.x = f29_out(p.x); r.y = f29_out(p.y); r.zz = f29_out(p.zz); r.zzz = f29_out(p.zzz); }
    for (Fq *f : {&r.x, &r.y, &r.zz, &r.zzz}) { reduce_once(*f); }
    G1Affine a = xyzz_to_affine(ref), b = xyzz_to_affine(r);
    if (!(a.x == b.x && a.y == b.y)) { if (bad < 3) printf("mismatch chain %d len %d\n", chain, len); bad++; }
  }
  printf("bad %d of 20000\n", bad);
  return bad != 0;
}
