/*
 * oracle.h -- plain-C CPU restatement of the twist-and-shout prover.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load liboracle.so, and only as the checker /
 * the timed CPU baseline -- never as part of the product path.
 *
 * It restates the reference algorithms *as written* (O(N^3) Lagrange
 * interpolation, per-term KZG commit, closure-driven sum-check that calls the
 * O(N*n) MLE evaluate at every hypercube point), so its run time is the
 * reference prover's algorithmic cost on this host.  See oracle.c for the
 * file:line citations.  Independent of the product arithmetic: 4 x u64 limbs
 * with unsigned __int128, where the GPU library uses 8 x u32 limbs.
 *
 * Data layout (same as arkworks in memory): Fr / Fq = uint64_t[4] little-endian
 * Montgomery form, R = 2^256.  G1 affine = uint64_t[8] (x, y), identity = all
 * zero words.
 */
#ifndef TNS_ORACLE_H
#define TNS_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_MAX_ROUNDS 40

typedef struct {
  uint64_t commitment[2][8];
  uint32_t num_rounds;
  uint32_t num_openings;
  uint64_t round_polynomials[ORC_MAX_ROUNDS][4][4];
  uint64_t final_evaluation[4];
  uint64_t opening_proofs[2][8];
  uint64_t final_evaluations[2][4];
  uint64_t opening_point[4];
  uint64_t sumcheck_challenges[ORC_MAX_ROUNDS][4];
} orc_proof;

/* field helpers (Montgomery limbs in/out) */
void orc_fr_from_u64(uint64_t v, uint64_t out[4]);
void orc_fr_to_canonical(const uint64_t a[4], uint64_t out[4]);
void orc_fr_from_canonical(const uint64_t a[4], uint64_t out[4]);
void orc_fr_mul(const uint64_t a[4], const uint64_t b[4], uint64_t out[4]);
void orc_fr_inv(const uint64_t a[4], uint64_t out[4]);

/* primitives */
void orc_chacha20_block(const uint32_t key[8], uint64_t counter, uint32_t out[16]);
uint64_t orc_siphash(const uint8_t *msg, size_t len, uint64_t k0, uint64_t k1, int c, int d);

/* src/utils.rs:79-131: tau, FS seed, and (optionally) the n_powers SRS points. */
size_t orc_setup_num_powers(unsigned log_size);
void orc_setup_params(unsigned log_size, uint64_t tau_out[4], uint8_t seed_out[32],
                      uint64_t *g1_powers_out /* nullable, n_powers*8 */);

/* src/polynomials.rs:301-352 over nodes 0..n-1 */
void orc_interpolate_consecutive(const uint64_t *y, size_t n, uint64_t *coeffs);
/* src/commitments.rs:162-180; returns 0 or 4 (Commitment error) */
int orc_commit(const uint64_t *g1_powers, size_t n_powers, const uint64_t *coeffs, size_t n,
               uint64_t out_affine[8]);
/* src/commitments.rs:182-199 */
int orc_open(const uint64_t *g1_powers, size_t n_powers, const uint64_t *coeffs, size_t n,
             const uint64_t z[4], uint64_t value[4], uint64_t proof_affine[8]);
void orc_commitment_hash(const uint64_t affine[8], uint64_t out[4]);
void orc_horner(const uint64_t *coeffs, size_t n, const uint64_t z[4], uint64_t out[4]);

/* src/polynomials.rs:85-161 */
void orc_mle_evaluate(const uint64_t *evals, unsigned nv, const uint64_t *point, uint64_t out[4]);
void orc_mle_partial_evaluate(const uint64_t *evals, unsigned nv, const uint64_t *fixed, unsigned k,
                              uint64_t *out);

/*
 * src/sumcheck.rs:56-110 with the closure f(x) = sum_t coeff_t * prod_{j<deg_t} T_{idx[t][j]}(x),
 * each T evaluated by the reference MLE evaluate at every point.
 * term_tables: n_terms*3 ints (unused slots = -1).  Returns 0 or 6 (SumCheck error).
 */
int orc_sumcheck_prove(const uint64_t *const *tables, int n_tables, unsigned nv,
                       const uint64_t *claimed_sum, int n_terms, const uint64_t *term_coeffs,
                       const int *term_tables, const uint8_t *transcript_prefix, size_t prefix_len,
                       uint64_t *rounds_out, uint64_t final_out[4], uint64_t *challenges_out);

/* Transcript challenge after absorbing `state` (src/utils.rs:172-192) */
void orc_transcript_challenge(const uint8_t *state, size_t len, uint64_t out[4]);

/* src/twist.rs:107-252.  addr/val/is_write: n_ops entries. Returns 0 or status. */
int orc_twist_prove(const uint64_t *g1_powers, size_t n_powers, size_t max_ops,
                    const uint64_t *addr, const uint64_t *val, const uint8_t *is_write,
                    size_t n_ops, orc_proof *out);
/* src/shout.rs:97-222 */
int orc_shout_prove(const uint64_t *g1_powers, size_t n_powers, size_t max_ops,
                    const uint64_t *entries, size_t n_entries, const uint64_t *indices,
                    size_t n_lookups, orc_proof *out);

#ifdef __cplusplus
}
#endif
#endif
