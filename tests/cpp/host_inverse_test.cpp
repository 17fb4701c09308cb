// CPU test (tests/test_host_field.py): the host binary extended-Euclid inverse (bn254.hpp inv_binary_host)
// against the Fermat chain a^(M-2) for Fr and Fq, 2000 random elements each plus 0 and 1.
#include "common.hpp"
#include <random>
#include <chrono>
using namespace tns;
template <class C> int check(const char *name) {
  std::mt19937_64 g(7);
  int bad = 0;
  double tb = 0, tf = 0;
  for (int it = 0; it < 2000; it++) {
    Fp<C> a;
    for (int i = 0; i < 8; i++) a.v[i] = (u32)g();
    a.v[7] &= 0x0fffffff;
    if (it == 0) a = Fp<C>::zero();
    if (it == 1) a = Fp<C>::one();
    auto t0 = std::chrono::steady_clock::now();
    Fp<C> x = inv_binary_host(a);
    auto t1 = std::chrono::steady_clock::now();
    u32 e[8]; u64 br = 2;
    for (int i = 0; i < 8; i++) { u64 d = (u64)C::M[i] - br; e[i] = (u32)d; br = (d >> 32) & 1; }
    Fp<C> y = pow_limbs(a, e);
    auto t2 = std::chrono::steady_clock::now();
    tb += std::chrono::duration<double>(t1 - t0).count(); tf += std::chrono::duration<double>(t2 - t1).count();
    Fp<C> r = x, q = y; reduce_once(r); reduce_once(q);
    if (!(r == q)) bad++;
  }
  printf("%s: %d mismatches of 2000; binary %.2f us, Fermat %.2f us per inverse\n", name, bad, tb / 2000 * 1e6, tf / 2000 * 1e6);
  return bad;
}
int main() { return check<FrCfg>("Fr") + check<FqCfg>("Fq"); }
