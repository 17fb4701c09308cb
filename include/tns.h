/*
 * tns.h -- C ABI of libtns, the MI355X (gfx950) twist-and-shout prover hot path.
 *
 * This is the drop-in boundary: the entry points a Rust `extern "C"` block (see
 * INTEGRATION.md) binds beneath the unchanged signatures of the reference crate
 * `twist-and-shout` (/root/reference).  Each function cites the reference
 * interface it replaces.
 *
 * Conventions
 *  - Field elements (Fr, Fq) are `uint64_t[4]`, little-endian, Montgomery form
 *    with R = 2^256: the in-memory layout of arkworks 0.4 `Fp256`, so a Rust
 *    `&[Fr]` can be passed as `*const u64` without conversion.
 *  - G1 affine inputs are `uint64_t[8]` = (x, y), Montgomery Fq; the all-zero
 *    pair encodes the identity.
 *  - G1 outputs are `uint64_t[12]` = arkworks `G1Projective` (Jacobian X, Y, Z),
 *    normalised: Z = 1 (Montgomery one) for finite points, (1, 1, 0) for the
 *    identity (ark-ec 0.4 `Projective::zero()`).
 *  - All pointers are caller-owned host memory, not retained after return.
 *    Every call is synchronous (stream-synchronised before return) and
 *    serialised per context; distinct contexts may be used from distinct threads.
 *  - Status codes mirror `TwistAndShoutError` (src/lib.rs:59-78); device
 *    failures are >= 100.  `tns_last_error()` returns a thread-local message.
 */
#ifndef TNS_H
#define TNS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  TNS_OK = 0,
  TNS_ERR_INVALID_PARAMETERS = 1, /* TwistAndShoutError::InvalidParameters */
  TNS_ERR_PROOF_GENERATION = 2,   /* ::ProofGeneration */
  TNS_ERR_PROOF_VERIFICATION = 3, /* ::ProofVerification */
  TNS_ERR_COMMITMENT = 4,         /* ::Commitment */
  TNS_ERR_POLYNOMIAL = 5,         /* ::Polynomial */
  TNS_ERR_SUMCHECK = 6,           /* ::SumCheck */
  TNS_ERR_DEVICE = 100,           /* HIP runtime failure */
  TNS_ERR_NO_DEVICE = 101,        /* no gfx950 device visible */
  TNS_ERR_OOM = 102               /* device allocation failed */
};

#define TNS_MAX_ROUNDS 40

typedef struct tns_ctx tns_ctx;
typedef struct tns_srs tns_srs;
typedef struct tns_transcript tns_transcript;

/* Output of setup_params (src/utils.rs:79-131). */
typedef struct {
  uint64_t log_size;
  uint64_t max_operations;  /* 1 << (log_size + 2)                    (src/utils.rs:80)      */
  uint64_t num_powers;      /* next_pow2(max_operations) + 1 SRS points (src/utils.rs:89-96) */
  uint64_t tau[4];          /* CommitmentParams.tau (Montgomery)      (src/utils.rs:84,107)  */
  uint8_t fiat_shamir_seed[32];                                   /* (src/utils.rs:101-102) */
} tns_params;

/*
 * One proof.  Twist (src/twist.rs:76-89): commitments = {address, value}.
 * Shout (src/shout.rs:64-79): commitments = {table, index}.  The trailing
 * fields are diagnostics the reference computes but does not return.
 */
typedef struct {
  uint64_t commitments[2][12];                      /* KZGCommitmentValue x2 */
  uint32_t num_rounds;                              /* SumCheckProof rounds = log2(padded ops) */
  uint32_t num_openings;                            /* 0 (no challenges) or 2 */
  uint64_t round_polynomials[TNS_MAX_ROUNDS][4][4]; /* SumCheckProof.round_polynomials */
  uint64_t final_evaluation[4];                     /* SumCheckProof.final_evaluation */
  uint64_t opening_proofs[2][12];                   /* Vec<KZGProof> */
  uint64_t final_evaluations[2][4];                 /* Vec<FieldElement> */
  /* diagnostics */
  uint64_t opening_point[4];                        /* challenges[0] */
  uint64_t sumcheck_challenges[TNS_MAX_ROUNDS][4];
  uint64_t final_mle_evals[3][4];                   /* MLE values at the sum-check point */
} tns_proof;

/* A degree <= 3 product term of a sum-check composition: coeff * prod T[tables[j]]
 * (tables[j] = -1 for unused slots). */
typedef struct {
  uint64_t coeff[4];
  int32_t tables[3];
  int32_t pad;
} tns_term;

/* ---------------------------------------------------------------- library */
const char *tns_last_error(void);
int tns_version(void);
/* Number of visible HIP devices (0 if none); never fails. */
int tns_device_count(void);

/* Identity and clock ratings of one visible device (hipDeviceProp_t), recorded beside
 * benchmark numbers so that a box's clocks can explain a difference between runs.  Not on
 * the reference's path (bench.py's device-state record, src/benchmarks.rs:26-28). */
typedef struct {
  char name[64];          /* marketing name */
  char arch[32];          /* gcnArchName, e.g. "gfx950:sramecc+:xnack-" */
  char pci_bus_id[32];    /* "DDDD:BB:DD.F", the sysfs name of the device */
  int32_t clock_khz;      /* peak shader clock (clockRate) */
  int32_t mem_clock_khz;  /* peak memory clock (memoryClockRate) */
  int32_t cu_count;       /* multiProcessorCount */
  int32_t pad;
  uint64_t total_mem;     /* bytes */
} tns_device_info;
int tns_device_info_get(int device, tns_device_info *out);

/* ---------------------------------------------------------------- context */
int tns_ctx_create(int device, tns_ctx **out);
/* tns_ctx_create with flags (0 = tns_ctx_create).  By default an MSM pair's accumulations run on
 * a least-priority stream and the context stream at the greatest priority, which orders the pair's
 * second sort behind the first accumulation (C4: -0.3-0.45 ms a proof).
 * TNS_CTX_NO_STREAM_PRIORITIES: every stream at the default priority -- for processes that share
 * one GPU, whose least-priority queues otherwise starve behind the other processes' (4 processes
 * on one GPU: 190 -> 330-360 ms a proof).  Same proofs either way; unknown flags ->
 * TNS_ERR_INVALID_PARAMETERS. */
#define TNS_CTX_NO_STREAM_PRIORITIES 1u
int tns_ctx_create_ex(int device, unsigned flags, tns_ctx **out);
void tns_ctx_destroy(tns_ctx *ctx);
int tns_ctx_synchronize(tns_ctx *ctx);

/* ---------------------------------------------------------------- setup / SRS */
/* setup_params(log_size) (src/utils.rs:79-131): derives tau and the FS seed from
 * ChaCha20Rng([42;32]) on the host and generates the `num_powers` G1 powers of tau
 * on the device.  *srs_out may be NULL to skip SRS generation. */
int tns_setup_params(tns_ctx *ctx, unsigned log_size, tns_params *out, tns_srs **srs_out);
/* Upload an externally built CommitmentParams.g1_powers (affine, n points). */
int tns_srs_upload(tns_ctx *ctx, const uint64_t *g1_affine, size_t n, tns_srs **out);
/* Copy points [0, n) of the SRS to host memory (affine uint64_t[8] each). */
int tns_srs_download(tns_ctx *ctx, const tns_srs *srs, uint64_t *g1_affine_out, size_t n);
/* Copy the points g1_powers[idx[t]], t < k, to host memory (affine uint64_t[8] each).  Every
 * index must lie in this SRS's share (all of g1_powers, or a shard's [first, first + held)):
 * spot checks of a large (or sharded) SRS without downloading it (CommitmentParams.g1_powers
 * is a public Vec the reference's own test reads, src/utils.rs:56, :283). */
int tns_srs_download_indices(tns_ctx *ctx, const tns_srs *srs, const uint64_t *idx, size_t k,
                             uint64_t *g1_affine_out);
/* The share of g1_powers this SRS holds: [first, first + held) (0 and tns_srs_len unsharded). */
int tns_srs_share(const tns_srs *srs, uint64_t *first, uint64_t *held);
size_t tns_srs_len(const tns_srs *srs);
void tns_srs_destroy(tns_srs *srs);
/* Attach the setup trapdoor kept in CommitmentParams.tau (src/utils.rs:60-61, :94-100)
 * to an uploaded SRS (tns_setup_params attaches it itself).  With it the SRS also
 * provides the Lagrange basis [L_j(tau)]G of the nodes {0..N-1}, which lets
 * Twist/Shout::prove commit to and open evaluation vectors without interpolating
 * them (same commitments and proofs).  tau: Montgomery-form Fr. */
int tns_srs_set_tau(tns_srs *srs, const uint64_t tau[4]);
/* Build (and cache in the SRS) the Lagrange basis for N = 2^k nodes ahead of the first
 * proof of that size; part of setup, not of proving.  TNS_ERR_INVALID_PARAMETERS when
 * the SRS has no tau or N is not a power of two. */
int tns_srs_prepare_lagrange(tns_ctx *ctx, tns_srs *srs, size_t n);
/* The same basis built from g1_powers[0..n) ALONE, for an SRS without tau (src/utils.rs:61, :107
 * mark tau test-only): a transposed remainder tree over the nodes' subproduct tree, ~1.5 n log^2 n
 * variable-base scalar multiplications on the device (tfree.hip; a one-time setup per (SRS, n) --
 * measured cost in DESIGN.md).  Cached in the SRS: Twist/Shout::prove then take the Lagrange route
 * on this SRS too.  n a power of two, g1_powers[0..n) held (unsharded). */
int tns_srs_prepare_lagrange_from_powers(tns_ctx *ctx, tns_srs *srs, size_t n);
/* Copy that basis ([L_j(tau)]G, j < n; built if needed) to host memory (affine uint64_t[8]
 * each): setup artefact for host-side provers (the CPU baseline of bench.py). */
int tns_srs_lagrange_download(tns_ctx *ctx, tns_srs *srs, size_t n, uint64_t *g1_affine_out);
/* Prove path selection: lagrange != 0 (default) commits/opens through the Lagrange
 * basis when the SRS has tau; 0 forces vector_to_polynomial + coefficient KZG
 * (src/twist.rs:151-163).  Both produce identical proofs. */
int tns_ctx_set_commit_basis(tns_ctx *ctx, int lagrange);
/* MSM over a fixed base (SRS, Lagrange basis): on != 0 (default) uses the base's
 * window-shifted table (built once, W copies of the points) so that every window shares
 * one bucket set; 0 forces the per-window bucket layout.  Same results.
 * MSM window tables (memory contract): a table is built the first time an MSM of >= 2^16 SRS
 * points / >= 2^12 Lagrange-basis points runs with tables on, and lives as long as its SRS:
 * W * n * 64 bytes for n points, W = ceil(255 / c) with the cost model's window c (C4's 2^24-node
 * basis: c = 22, W = 12, 12.9 GB; C2's 2^20 + 1 SRS points: c = 20, W = 13, 0.87 GB).  If the
 * device cannot hold it, the MSM runs without it (per-window buckets: same result, slower) and
 * nothing is cached -- no error is returned for a table.  Setting 0 here before the first MSM
 * keeps every table from being built. */
int tns_ctx_set_msm_tables(tns_ctx *ctx, int on);
/* Drop-in provers (tns_twist_prove on host buffers): the value vector crosses PCIe in `chunks`
 * equal node ranges (1..64, default 4), each committed by its own MSM as soon as it lands, so only
 * the last range's MSM follows the link (C4: commit phase 19.0 -> 15.5 ms at 4).  Same proofs
 * for every setting; out of range -> TNS_ERR_INVALID_PARAMETERS.  The library reads no tuning
 * from the environment: this, the two setters above and tns_ctx_create_ex's flags are its
 * whole tuning surface. */
int tns_ctx_set_upload_chunks(tns_ctx *ctx, int chunks);

/* ---------------------------------------------------------------- KZG (src/commitments.rs) */
/* CommitmentScheme::commit for KZGCommitment (src/commitments.rs:162-180).
 * n > srs_len -> TNS_ERR_COMMITMENT ("Polynomial degree exceeds setup size"). */
int tns_kzg_commit(tns_ctx *ctx, const tns_srs *srs, const uint64_t *coeffs, size_t n,
                   uint64_t out_proj[12]);
/* CommitmentScheme::open (src/commitments.rs:182-199): value = P(z) (Horner,
 * :305-313) and proof = commit((P - v) / (x - z)) (:317-375). n <= 1 -> identity proof. */
int tns_kzg_open(tns_ctx *ctx, const tns_srs *srs, const uint64_t *coeffs, size_t n,
                 const uint64_t z[4], uint64_t value[4], uint64_t proof_proj[12]);
/* commit(vector_to_polynomial(evals)) and open(vector_to_polynomial(evals), z) in one
 * step (src/polynomials.rs:248-262 then src/commitments.rs:162-199), as Twist/Shout::prove
 * do: through the SRS's Lagrange basis when it has tau, else by interpolation (which needs
 * n to be a power of two, as the provers pad to, src/twist.rs:141). */
int tns_kzg_commit_evals(tns_ctx *ctx, const tns_srs *srs, const uint64_t *evals, size_t n,
                         uint64_t out_proj[12]);
int tns_kzg_open_evals(tns_ctx *ctx, const tns_srs *srs, const uint64_t *evals, size_t n,
                       const uint64_t z[4], uint64_t value[4], uint64_t proof_proj[12]);
/* KZGVectorCommitment::open (src/commitments.rs:440-471): the opening of the vector's
 * interpolant at the node `index` (value = vec[index]); commit = tns_kzg_commit_evals (any n
 * when the SRS carries tau); verify = tns_kzg_verify at z = index.  index >= n ->
 * TNS_ERR_COMMITMENT ("Index out of bounds"). */
int tns_vc_open(tns_ctx *ctx, const tns_srs *srs, const uint64_t *vec, size_t n, size_t index, uint64_t value[4],
                uint64_t proof_proj[12]);
/* KZGCommitmentValue::hash (src/commitments.rs:73-84).  Host only. */
int tns_commitment_hash(const uint64_t proj[12], uint64_t out[4]);
/* Raw MSM: sum_i scalars[i] * points[i] over the first n SRS points. */
int tns_msm(tns_ctx *ctx, const tns_srs *srs, const uint64_t *scalars, size_t n,
            uint64_t out_proj[12]);

/* ---------------------------------------------------------------- polynomials */
/* poly_utils::lagrange_interpolate over the nodes 0..n-1 (src/polynomials.rs:301-352,
 * as called by vector_to_polynomial, src/twist.rs:307-315): the n monomial
 * coefficients of the unique interpolant, computed exactly in O(n log^2 n). */
int tns_interpolate_consecutive(tns_ctx *ctx, const uint64_t *y, size_t n, uint64_t *coeffs);
/* MultilinearExtension::evaluate (src/polynomials.rs:85-103); variable j <-> index bit j.
 * evals holds n_evals <= 2^nv entries (the reference struct's `evaluations`); missing
 * entries are zero.  n_evals > 2^nv -> TNS_ERR_INVALID_PARAMETERS (the reference's basis
 * reads only the low nv index bits, so callers fold entry i into i mod 2^nv first). */
int tns_mle_evaluate(tns_ctx *ctx, const uint64_t *evals, size_t n_evals, unsigned nv,
                     const uint64_t *point, uint64_t out[4]);
/* MultilinearExtension::partial_evaluate (src/polynomials.rs:126-161): binds the
 * first k (least-significant) variables; out has 2^(nv-k) entries.  evals as above. */
int tns_mle_partial_evaluate(tns_ctx *ctx, const uint64_t *evals, size_t n_evals, unsigned nv,
                             const uint64_t *fixed, unsigned k, uint64_t *out);

/* ---------------------------------------------------------------- transcript (src/utils.rs:134-204) */
tns_transcript *tns_transcript_new(const uint8_t seed[32]);
void tns_transcript_free(tns_transcript *t);
void tns_transcript_append_field_element(tns_transcript *t, const uint8_t *label, size_t label_len,
                                         const uint64_t x[4]);
void tns_transcript_append_field_elements(tns_transcript *t, const uint8_t *label,
                                          size_t label_len, const uint64_t *xs, size_t n);
void tns_transcript_challenge_field_element(tns_transcript *t, const uint8_t *label,
                                            size_t label_len, uint64_t out[4]);

/* ---------------------------------------------------------------- sum-check (src/sumcheck.rs:56-110) */
/* SumCheck::prove for the closure x -> sum_t coeff_t * prod_j MLE(T_{t,j})(x) over n_tables
 * MLE tables of 2^nv entries each (degree <= 3 per variable, as the reference's 4-point
 * round interpolation assumes; at most 4 tables and 64 terms, terms over the same tables
 * combine).  rounds_out: nv x 4 Fr; challenges_out: nv Fr (nullable). */
int tns_sumcheck_prove(tns_ctx *ctx, const uint64_t *const *tables, int n_tables, unsigned nv,
                       const uint64_t claimed_sum[4], const tns_term *terms, int n_terms,
                       tns_transcript *transcript, uint64_t *rounds_out, uint64_t final_out[4],
                       uint64_t *challenges_out);
/* The composition's sum over {0,1}^nv (the honest claimed_sum) on device tables. */
int tns_composition_sum_device(tns_ctx *ctx, const uint64_t *const *d_tables, int n_tables, unsigned nv,
                               const tns_term *terms, int n_terms, uint64_t out[4]);
/* The same on tables already resident in HBM (device pointers, only read). */
int tns_sumcheck_prove_device(tns_ctx *ctx, const uint64_t *const *d_tables, int n_tables, unsigned nv,
                              const uint64_t claimed_sum[4], const tns_term *terms, int n_terms,
                              tns_transcript *transcript, uint64_t *rounds_out, uint64_t final_out[4],
                              uint64_t *challenges_out);

/* ---------------------------------------------------------------- protocols */
/* Twist::prove (src/twist.rs:107-252).  The MemoryTrace's operations as SoA:
 * addr[i] (usize address), value[i] (Fr), is_write[i] (1 = Write, 0 = Read). */
int tns_twist_prove(tns_ctx *ctx, const tns_srs *srs, const tns_params *params,
                    const uint64_t *addr, const uint64_t *value, const uint8_t *is_write,
                    size_t n_ops, tns_proof *out);
/* Shout::prove (src/shout.rs:97-222).  LookupTable.entries (Fr) and the lookup
 * indices (usize). */
int tns_shout_prove(tns_ctx *ctx, const tns_srs *srs, const tns_params *params,
                    const uint64_t *entries, size_t n_entries, const uint64_t *indices,
                    size_t n_lookups, tns_proof *out);

/* ---------------------------------------------------------------- device-resident inputs */
/* The same provers on inputs already resident in HBM (device pointers, e.g. from
 * tns_buffer_upload): the steady-state serving path, no PCIe in the prove. */
typedef struct tns_buffer tns_buffer;
int tns_buffer_upload(tns_ctx *ctx, const void *host, size_t bytes, tns_buffer **out);
void *tns_buffer_device_ptr(const tns_buffer *buf);
/* Copy the first `bytes` of the buffer back to host memory. */
int tns_buffer_download(const tns_buffer *buf, void *host, size_t bytes);
void tns_buffer_free(tns_buffer *buf);
int tns_twist_prove_device(tns_ctx *ctx, const tns_srs *srs, const tns_params *params,
                           const uint64_t *d_addr, const uint64_t *d_value,
                           const uint8_t *d_is_write, size_t n_ops, tns_proof *out);
int tns_shout_prove_device(tns_ctx *ctx, const tns_srs *srs, const tns_params *params,
                           const uint64_t *d_entries, size_t n_entries, const uint64_t *d_indices,
                           size_t n_lookups, tns_proof *out);
/* KZGCommitment::commit / MSM on device-resident scalars. */
int tns_msm_device(tns_ctx *ctx, const tns_srs *srs, const uint64_t *d_scalars, size_t n,
                   uint64_t out_proj[12]);

/* ---------------------------------------------------------------- verifiers (host)
 * CommitmentVerificationKey (src/utils.rs:64-75, :104-112): G1 generator, G2 generator and
 * tau*G2, affine Montgomery limbs; G2 coordinates as x.c0, x.c1, y.c0, y.c1 (Fq2 = Fq[u]/(u^2+1)),
 * identity = all zeros. */
typedef struct tns_vk {
  uint64_t g1[8];
  uint64_t g2[16];
  uint64_t g2_tau[16];
} tns_vk;
int tns_verifier_key(const tns_params *params, tns_vk *out);
/* KZGCommitment::verify (src/commitments.rs:201-228): e(C - v G1, G2) == e(pi, tau G2 - z G2). */
int tns_kzg_verify(const tns_vk *vk, const uint64_t commitment_proj[12], const uint64_t z[4],
                   const uint64_t value[4], const uint64_t proof_proj[12], int *ok);
/* KZGCommitment::batch_verify (src/commitments.rs:230-301), the reference's equation as written;
 * arrays of n entries (commitments/proofs uint64_t[12] each, points/values uint64_t[4]). */
int tns_kzg_batch_verify(const tns_vk *vk, size_t n, const uint64_t *commitments_proj, const uint64_t *points,
                         const uint64_t *values, const uint64_t *proofs_proj, int *ok);
/* Twist::verify / Shout::verify (src/twist.rs:255-304, src/shout.rs:225-274) on a proof of
 * tns_twist_prove / tns_shout_prove; *ok = 1 valid, 0 invalid. */
int tns_twist_verify(const tns_vk *vk, const tns_proof *proof, int *ok);
int tns_shout_verify(const tns_vk *vk, const tns_proof *proof, int *ok);
/* Bn254::pairing(P, Q) (arkworks optimal ate): 12 Fq (Montgomery), tower order
 * c0.c0.c0, c0.c0.c1, c0.c1.c0, ..., c1.c2.c1.  Test / interop utility. */
int tns_pairing(const uint64_t g1_affine[8], const uint64_t g2_affine[16], uint64_t out[48]);
/* k * Q on G2 for a canonical scalar k (uint64_t[4]). */
int tns_g2_mul(const uint64_t g2_affine[16], const uint64_t k_canonical[4], uint64_t out[16]);

/* ---------------------------------------------------------------- wire format
 * CanonicalSerialize of KZGCommitmentValue / KZGProof (src/commitments.rs:94-154) = the G1
 * point's ark-serialize 0.4 encoding: 32 bytes (compressed: x LE, flags 0x80 y-negative /
 * 0x40 infinity in the last byte) or 64 bytes (x, y).  Fr: 32 bytes LE.  Proofs
 * (TwistProof / ShoutProof, src/twist.rs:76-89, src/shout.rs:64-79): fields in order, Vec as
 * u64 LE length + elements.  Deserialisation validates (field range, curve membership). */
int tns_g1_serialize(const uint64_t proj[12], int compressed, uint8_t *out);
int tns_g1_deserialize(const uint8_t *in, int compressed, uint64_t proj_out[12]);
int tns_proof_serialize(const tns_proof *proof, int compressed, uint8_t *out, size_t cap, size_t *len);
int tns_proof_deserialize(const uint8_t *in, size_t len, int compressed, tns_proof *out);

/* ---------------------------------------------------------------- one proof across GPUs
 * SURVEY 8(e) / BASELINE C5: the evaluation vectors and the SRS of ONE Twist/Shout proof
 * sharded over `size` ranks (one process -- or one tns_ctx -- per GPU).  Rank r holds the
 * contiguous slice [r N/size, (r+1) N/size) of the padded length-N vectors and the matching
 * slice of the Lagrange basis; the exchange steps are allgathers of partial MSM sums,
 * barycentric partials and one folded value per MLE table (a few hundred bytes per step).
 * Every rank returns the same proof, identical to the unsharded prover's.  size must be a
 * power of two <= N; the SRS must carry tau (setup_params / tns_srs_set_tau). */
typedef struct tns_comm tns_comm;
/* allgather: place every rank's `bytes` from `send`, in rank order, into `recv`
 * (size * bytes); return 0 on success. */
typedef int (*tns_allgather_fn)(void *user, const void *send, size_t bytes, void *recv);
/* RCCL communicator (ncclAllGather on the context's stream).  Rank 0 calls
 * tns_comm_unique_id and the launcher broadcasts the 128 bytes. */
int tns_comm_unique_id(uint8_t uid[128]);
int tns_comm_create(tns_ctx *ctx, int rank, int size, const uint8_t uid[128], tns_comm **out);
/* Communicator over any host-side transport. */
int tns_comm_create_callback(int rank, int size, tns_allgather_fn fn, void *user, tns_comm **out);
void tns_comm_destroy(tns_comm *comm);
/* rank and size the communicator was created with, the rank count its transport reports
 * (ncclCommCount for RCCL, else size) and its kind: 0 one rank, 1 host callback, 2 RCCL. */
int tns_comm_info(const tns_comm *comm, int *rank, int *size, int *seen_size, int *kind);
/* The communicator's allgather on its own (self-test / launcher use); ctx may be NULL for a
 * callback communicator. */
int tns_comm_allgather(tns_ctx *ctx, tns_comm *comm, const void *send, size_t bytes, void *recv);
/* Deadline of one exchange step (default 600 s).  RCCL: the collective is polled on the
 * context stream and the communicator is aborted past the deadline; a host callback enforces
 * its own deadline and returns non-zero.  Either way the prove call fails with TNS_ERR_DEVICE and
 * a message naming this rank, the exchange step number and what it carried. */
int tns_comm_set_timeout(tns_comm *comm, double seconds);
/* out = {exchange steps so far, their total seconds, the longest one's seconds, the deadline}
 * (multi-rank communicators; timed on the host around each allgather). */
int tns_comm_stats(const tns_comm *comm, double out[4]);
/* tns_comm_stats + {bytes this rank sent over all exchange steps, the largest step's bytes}. */
int tns_comm_stats_ex(const tns_comm *comm, double out[6]);
/* Build (and cache) rank `rank` of `size`'s slice of the Lagrange basis for N = 2^k nodes
 * ahead of the first sharded proof of that size (setup, like tns_srs_prepare_lagrange). */
int tns_srs_prepare_lagrange_shard(tns_ctx *ctx, tns_srs *srs, size_t n, int rank, int size);
/* setup_params for rank `rank` of `size`: the same params/tau as tns_setup_params, with the
 * SRS holding only its contiguous share of g1_powers (the "SRS shard generated locally from
 * tau"); tns_srs_len still reports the full length. */
int tns_setup_params_shard(tns_ctx *ctx, unsigned log_size, int rank, int size, tns_params *out,
                           tns_srs **srs_out);
/* KZGCommitment::commit (src/commitments.rs:162-180) of n_total coefficients sharded over the
 * ranks (the C2 MSM at N GPUs): rank r holds coefficients [r N/size, r N/size + n_local) on the
 * device (N = next_pow2(n_total); n_local = that slice's length) and an SRS share covering them
 * (tns_setup_params_shard splits 2^k + 1 powers on those boundaries); one partial MSM per rank,
 * an allgather of the 96-byte partials.  Every rank returns the whole commitment.
 * Restriction: the slices must lie in the ranks' SRS shares, which follow the setup's 2^k
 * boundaries, so next_pow2(n_total) must equal that 2^k (e.g. n_total = 2^20 over
 * setup_params_shard(18)); any other n_total fails with TNS_ERR_INVALID_PARAMETERS (an unsharded
 * tns_msm / tns_kzg_commit takes every length up to the SRS's). */
int tns_msm_sharded(tns_ctx *ctx, const tns_srs *srs, tns_comm *comm, const uint64_t *d_scalars, size_t n_local,
                    uint64_t n_total, uint64_t out_proj[12]);
/* Twist::prove of a trace of n_total operations whose operations
 * [rank * N/size, rank * N/size + n_local) (N = next_pow2(n_total)) this rank holds on the
 * device; n_local must be that slice's length (0 for ranks past the end). */
int tns_twist_prove_sharded(tns_ctx *ctx, const tns_srs *srs, const tns_params *params, tns_comm *comm,
                            const uint64_t *d_addr, const uint64_t *d_value, const uint8_t *d_is_write,
                            size_t n_local, uint64_t n_total, tns_proof *out);
/* Shout::prove with the table (n_entries_total, padded T) and the lookup indices
 * (n_lookups_total, padded M) sliced the same way: entries [rank*T/size, +n_entries_local),
 * indices [rank*M/size, +n_lookups_local). */
int tns_shout_prove_sharded(tns_ctx *ctx, const tns_srs *srs, const tns_params *params, tns_comm *comm,
                            const uint64_t *d_entries, size_t n_entries_local, uint64_t n_entries_total,
                            const uint64_t *d_indices, size_t n_lookups_local, uint64_t n_lookups_total,
                            tns_proof *out);

/* ---------------------------------------------------------------- kernel timing */
/* HIP-event timing of the named stages on the context stream ("msm_accumulate",
 * "msm_sort", "msm_digits", "msm_reduce", "ntt_stage", "ntt_lds", "ntt_pointwise",
 * "interp_tile", "sumcheck_round", "open_scan").  Enabling resets the totals and the stage
 * filter of tns_profile_only (call that after enabling). */
int tns_profile_enable(tns_ctx *ctx, int on);
/* Restrict the timing to one stage (NULL or "": every stage).  Each timed stage costs two HIP
 * events per launch; the bench times only its roofline kernel inside the timed steps. */
int tns_profile_only(tns_ctx *ctx, const char *stage);
int tns_profile_read(tns_ctx *ctx, const char *stage, double *total_ms, uint64_t *launches,
                     double *algorithmic_bytes);
/* out = {summed launch ms, launches, algorithmic bytes, operations (msm_accumulate: mixed
 * additions), busy ms (union of the launch intervals: stages of the two MSM lanes overlap)} */
int tns_profile_read_ex(tns_ctx *ctx, const char *stage, double out[5]);
/* The shader clock the device holds under a full integer-VALU load shaped like the MSM
 * accumulation (chains of Montgomery products on every SIMD) for about `ms` milliseconds:
 * per workgroup, delta s_memtime / delta s_memrealtime x 100 MHz (the in-kernel clock of
 * MI355X_MICROARCH.md's DVFS notes).  out = {median MHz, min MHz, max MHz, kernel ms}.
 * A diagnostic beside benchmark numbers (VALU-bound kernels scale with it), not proving work. */
int tns_clock_probe(tns_ctx *ctx, double ms, double out[4]);

/* ---------------------------------------------------------------- host utilities (no device) */
/* Batch conversions between integers and Montgomery-form Fr / Fq (multi-threaded). */
void tns_fr_from_u64(const uint64_t *in, size_t n, uint64_t *out_mont);
void tns_fr_from_canonical(const uint64_t *in, size_t n, uint64_t *out_mont);
void tns_fr_to_canonical(const uint64_t *in_mont, size_t n, uint64_t *out);
void tns_fq_to_canonical(const uint64_t *in_mont, size_t n, uint64_t *out);
/* n successive `Fr::rand` draws (ark-ff 0.4.2 UniformRand) from ChaCha20Rng::from_seed(seed)
 * -- the synthetic scalars of the C2 MSM configuration (seed [7;32]). */
void tns_fr_rand_batch(const uint8_t seed[32], size_t n, uint64_t *out_mont);
/* The synthetic read/write trace of ProtocolBenchmarks (src/benchmarks.rs:88-99):
 * op i writes Fr(42 i) to i % memory_size when i % 3 == 0, else reads (i / 2) % memory_size
 * and records the current memory value.  value_u64 holds the values as integers. */
int tns_bench_trace(size_t memory_size, size_t n_ops, uint64_t *addr, uint64_t *value_u64,
                    uint8_t *is_write);
/* Operations [first, first + count) of the n_total-operation ProtocolBenchmarks trace (the
 * memory state is replayed from operation 0): one rank's slice of a sharded trace. */
int tns_bench_trace_slice(size_t memory_size, uint64_t n_total, uint64_t first, size_t count, uint64_t *addr,
                          uint64_t *value, uint8_t *is_write);

/* Wall-clock breakdown of the last prove on this context (milliseconds):
 * [0] H2D, [1] interpolation, [2] commit MSMs, [3] sum-check, [4] open, [5] total. */
int tns_last_prove_timing(tns_ctx *ctx, double out_ms[6]);

#ifdef __cplusplus
}
#endif
#endif /* TNS_H */
