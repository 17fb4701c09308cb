/*
 * fastcpu.h -- the fast CPU baseline (fastcpu.c): Twist::prove with the MI355X path's
 * algorithms on host threads.  BASELINE / TEST INFRASTRUCTURE ONLY (see oracle.h).
 * Layouts as in oracle.h (uint64_t[4] Montgomery field elements, uint64_t[8] affine G1).
 */
#ifndef TNS_FASTCPU_H
#define TNS_FASTCPU_H
#include <stddef.h>
#include <stdint.h>

#include "oracle.h"

#ifdef __cplusplus
extern "C" {
#endif

/* barycentric weights w_j = (-1)^(N-1-j) / (j! (N-1-j)!) of the nodes 0..N-1 (N x 4) */
void fc_bary_weights(size_t N, uint64_t *w);
/* [L_j(tau)]G, j < N (N x 8), by scalar multiplication -- small N (tests) */
void fc_lagrange_basis(const uint64_t tau[4], size_t N, uint64_t *out);
/* f0(x), f1(x) for two vectors of N evaluations on the nodes 0..N-1 (Montgomery, N x 4; y1 may
 * be y0) by the barycentric formula in O(N) on `threads` host threads, and ell(x) = prod (x - j).
 * Returns 1 when x is a node.  Size-independent parity checks (C = f(tau) G, pi (tau - z) = C - v G). */
int fc_bary_eval2(const uint64_t *bary_w, const uint64_t *y0, const uint64_t *y1, size_t N, const uint64_t x[4],
                  int threads, uint64_t f0[4], uint64_t f1[4], uint64_t ell[4]);
/* k G1 (k Montgomery Fr) and k P (P affine), affine out (identity = zeros) */
void fc_g1_mul_gen(const uint64_t k[4], uint64_t out[8]);
void fc_g1_mul(const uint64_t aff[8], const uint64_t k[4], uint64_t out[8]);
/* Twist::prove of n_ops operations (N = next_pow2(n_ops) >= 2): addr as u64, val Montgomery
 * Fr, is_write bytes; lagrange = [L_j(tau)]G and bary_w = fc_bary_weights(N).  threads: host
 * threads to use.  Returns 0, 1 (InvalidParameters) or 2 (opening point on a node). */
int fc_twist_prove(const uint64_t *lagrange, const uint64_t *bary_w, size_t N, size_t max_ops,
                   const uint64_t *addr, const uint64_t *val, const uint8_t *is_write, size_t n_ops,
                   int threads, orc_proof *out);

/* SumCheck::prove (src/sumcheck.rs:56-110) for the composition sum_t c_t prod_j T[tt[3t+j]]
 * (tt = -1 for unused slots, <= 4 tables of 2^nv Montgomery Fr) with O(N)-per-round table folds
 * on `threads` host threads; transcript = prefix bytes then the rounds.  Same outputs and status
 * (0, 1 bad arguments, 6 round check failed) as orc_sumcheck_prove. */
int fc_sumcheck_prove(const uint64_t *const *tables, int n_tables, unsigned nv, const uint64_t claimed[4],
                      int n_terms, const uint64_t *term_coeffs, const int *term_tables, const uint8_t *prefix,
                      size_t prefix_len, int threads, uint64_t *rounds_out, uint64_t final_out[4],
                      uint64_t *challenges_out);
/* sum over {0,1}^nv of that composition (the honest claimed sum) */
void fc_composition_sum(const uint64_t *const *tables, unsigned nv, int n_terms, const uint64_t *term_coeffs,
                        const int *term_tables, int threads, uint64_t out[4]);

#ifdef __cplusplus
}
#endif
#endif
