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

// All threads of the block run stages [0, lh_hi] (DIF: high to low; DIT: low to high)
// on `len` LDS elements holding independent transforms of size >= 2^(lh_hi+1).
template <bool INV>
__device__ __forceinline__ void lds_ntt(Fr *buf, unsigned len, int lh_hi, const Fr *__restrict__ TW) {
  const unsigned nbf = len >> 1;
  if (!INV) {
    for (int lh = lh_hi; lh >= 0; lh--) {
      const uint32_t h = 1u << lh;
      for (unsigned q = threadIdx.x; q < nbf; q += blockDim.x) {
        const uint32_t k = q & (h - 1);
        const uint32_t i0 = ((q >> lh) << (lh + 1)) | k, i1 = i0 + h;
        Fr a = buf[i0], b = buf[i1];
        buf[i0] = add(a, b);
        buf[i1] = mul(sub(a, b), ntt_tw(TW, lh, k, false));
      }
      __syncthreads();
    }
  } else {
    for (int lh = 0; lh <= lh_hi; lh++) {
      const uint32_t h = 1u << lh;
      for (unsigned q = threadIdx.x; q < nbf; q += blockDim.x) {
        const uint32_t k = q & (h - 1);
        const uint32_t i0 = ((q >> lh) << (lh + 1)) | k, i1 = i0 + h;
        Fr a = buf[i0], b = mul(buf[i1], ntt_tw(TW, lh, k, true));
        buf[i0] = add(a, b);
        buf[i1] = sub(a, b);
      }
      __syncthreads();
    }
  }
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
