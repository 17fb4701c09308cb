// ntt.hpp -- number-theoretic transforms over BN254 Fr for gfx950 (shared device helpers).
//
// Forward = decimation-in-frequency (natural order in, bit-reversed out); inverse =
// decimation-in-time (bit-reversed in, natural out), unscaled.  Pointwise products of
// two forward transforms are taken in bit-reversed order, so no permutation pass exists.
//
// Twiddles live in one stage-major table: TW[h + k] = w_{2h}^k for h = 2^lh, k < h
// (2^L entries cover every stage lh < L).  A stage's twiddles are contiguous, so the
// k-consecutive lanes of a pass read consecutive 32-byte entries (L2-resident; the
// table for 2^25 is 1 GiB of HBM but each pass touches only its stages' slices).
#pragma once
#include "common.hpp"

namespace tns {

// w_{2h}^k (forward) or w_{2h}^-k = -w_{2h}^(h-k) (inverse)
__device__ __forceinline__ Fr ntt_tw(const Fr *__restrict__ TW, unsigned lh, uint32_t k, bool inv_dir) {
  const size_t h = (size_t)1 << lh;
  if (!inv_dir || k == 0) return TW[h + k];
  return neg(TW[2 * h - k]);
}

// ---------------------------------------------------------------- LDS stage engine
// A tile in LDS is `rows` x COLS elements, buf[j * COLS + c]; row j of column c is the
// global element  base + (j << lo) + colbase + c  of a transform, so local stage ll is the
// global stage lh = lo + ll and its twiddle index is k = (j mod 2^ll) << lo | colbase + c.
// Stages run two at a time (radix-4: 4 LDS reads, 3 twiddles, 4 multiplies, 4 LDS writes
// and one barrier per two stages); an odd count does one radix-2 stage first (DIF: the
// top stage) or last (DIT: the top stage).

// SUB = true: a pure size-`rows` sub-DFT per column (twiddle index kl, no column term) --
// the four-step form used by the strided passes, whose column term is applied separately.
template <bool INV, int COLS, bool SUB = false>
__device__ __forceinline__ void lds_radix2(Fr *buf, unsigned rows, int ll, unsigned lo, uint32_t colbase,
                                           const Fr *__restrict__ TW) {
  const unsigned d = 1u << ll, units = (rows >> 1) * COLS;
  for (unsigned q = threadIdx.x; q < units; q += blockDim.x) {
    const unsigned c = q % COLS, jq = q / COLS;
    const unsigned kl = jq & (d - 1);
    const unsigned j0 = ((jq >> ll) << (ll + 1)) | kl;
    const uint32_t k = SUB ? kl : ((uint32_t)kl << lo) + colbase + c;
    const Fr w = ntt_tw(TW, SUB ? ll : lo + ll, k, INV);
    const unsigned i0 = j0 * COLS + c, i1 = i0 + d * COLS;
    Fr a = buf[i0], b = buf[i1];
    if (!INV) {
      buf[i0] = add(a, b);
      buf[i1] = mul(sub(a, b), w);
    } else {
      b = mul(b, w);
      buf[i0] = add(a, b);
      buf[i1] = sub(a, b);
    }
  }
  __syncthreads();
}

// local stages (ll, ll - 1), quarter distance d = 2^(ll-1)
template <bool INV, int COLS, bool SUB = false>
__device__ __forceinline__ void lds_radix4(Fr *buf, unsigned rows, int ll, unsigned lo, uint32_t colbase,
                                           const Fr *__restrict__ TW) {
  const unsigned d = 1u << (ll - 1), units = (rows >> 2) * COLS;
  const unsigned lo_e = SUB ? 0 : lo;
  for (unsigned q = threadIdx.x; q < units; q += blockDim.x) {
    const unsigned c = q % COLS, jq = q / COLS;
    const unsigned kl = jq & (d - 1);
    const unsigned j0 = (jq >> (ll - 1)) * 4 * d + kl;
    const uint32_t k = SUB ? kl : ((uint32_t)kl << lo) + colbase + c;
    // twiddles: stage lh = lo+ll at k and k + d<<lo; stage lh-1 at k
    const Fr w1 = ntt_tw(TW, lo_e + ll, k, INV);
    const Fr w2 = ntt_tw(TW, lo_e + ll, k + ((uint32_t)d << lo_e), INV);
    const Fr w3 = ntt_tw(TW, lo_e + ll - 1, k, INV);
    const unsigned i0 = j0 * COLS + c, s = d * COLS;
    Fr x0 = buf[i0], x1 = buf[i0 + s], x2 = buf[i0 + 2 * s], x3 = buf[i0 + 3 * s];
    if (!INV) {
      Fr a0 = add(x0, x2), a2 = mul(sub(x0, x2), w1);
      Fr a1 = add(x1, x3), a3 = mul(sub(x1, x3), w2);
      buf[i0] = add(a0, a1);
      buf[i0 + s] = mul(sub(a0, a1), w3);
      buf[i0 + 2 * s] = add(a2, a3);
      buf[i0 + 3 * s] = mul(sub(a2, a3), w3);
    } else {
      Fr t1 = mul(x1, w3), t3 = mul(x3, w3);
      Fr a0 = add(x0, t1), a1 = sub(x0, t1), a2 = add(x2, t3), a3 = sub(x2, t3);
      Fr u2 = mul(a2, w1), u3 = mul(a3, w2);
      buf[i0] = add(a0, u2);
      buf[i0 + 2 * s] = sub(a0, u2);
      buf[i0 + s] = add(a1, u3);
      buf[i0 + 3 * s] = sub(a1, u3);
    }
  }
  __syncthreads();
}

// local stages [0, ll_hi] on a rows x COLS tile (DIF high -> low, DIT low -> high)
template <bool INV, int COLS, bool SUB = false>
__device__ __forceinline__ void lds_stages(Fr *buf, unsigned rows, int ll_hi, unsigned lo, uint32_t colbase,
                                           const Fr *__restrict__ TW) {
  const int n = ll_hi + 1;
  if (!INV) {
    int ll = ll_hi;
    if (n & 1) {
      lds_radix2<false, COLS, SUB>(buf, rows, ll, lo, colbase, TW);
      ll--;
    }
    for (; ll >= 1; ll -= 2) lds_radix4<false, COLS, SUB>(buf, rows, ll, lo, colbase, TW);
  } else {
    int ll = 1;
    for (; ll <= ll_hi - (n & 1); ll += 2) lds_radix4<true, COLS, SUB>(buf, rows, ll, lo, colbase, TW);
    if (n & 1) lds_radix2<true, COLS, SUB>(buf, rows, ll_hi, lo, colbase, TW);
  }
}

// All threads of the block run stages [0, lh_hi] (DIF: high to low; DIT: low to high)
// on `len` contiguous LDS elements holding independent transforms of size >= 2^(lh_hi+1).
template <bool INV>
__device__ __forceinline__ void lds_ntt(Fr *buf, unsigned len, int lh_hi, const Fr *__restrict__ TW) {
  lds_stages<INV, 1>(buf, len, lh_hi, 0, 0, TW);
}

// host entry points (ntt.hip)
const Fr *ntt_twiddles(Ctx *c, unsigned L);  // ensure stages < L; returns TW
// nb contiguous transforms of size 2^s (forward DIF or inverse DIT, unscaled)
void ntt_blocks(Ctx *c, Fr *x, unsigned s, size_t nb, bool inverse);
// x <- INTT(NTT(x) .* w) per block (w: a forward transform of size 2^s in bit-reversed
// order, pre-scaled by 2^-s): a cyclic convolution in 2 + 2*ceil((s-10)/7) HBM passes.
void ntt_conv_blocks(Ctx *c, Fr *x, unsigned s, size_t nb, const Fr *w);
Fr fr_root_of_unity(unsigned log_order);

}  // namespace tns
