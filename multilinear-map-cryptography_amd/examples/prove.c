/* prove.c -- a plain C host of the drop-in boundary (include/tns.h), no Python, no torch: the
 * calls a Rust binding of Twist::prove / Shout::prove makes (INTEGRATION.md sections 1 and 2b).
 *
 *   prove twist [log_size [n_ops [memory_size [reps]]]]         defaults 8 256 2^log_size 1
 *   prove shout [log_size [table_size [n_lookups [reps]]]]      defaults 8 256 256 1
 *
 * twist: setup_params(log_size) (src/utils.rs:79-131), the ProtocolBenchmarks trace of n_ops
 *   operations (src/benchmarks.rs:88-99), Twist::prove on host buffers (src/twist.rs:107-252,
 *   PCIe included), Twist::verify (src/twist.rs:255-304).
 * shout: the ProtocolBenchmarks lookup workload (src/benchmarks.rs:167-177): a table of squares
 *   i^2, lookups of index i % table_size; Shout::prove (src/shout.rs:97-222), Shout::verify
 *   (src/shout.rs:225-274).
 * Prints one JSON line {"ok", "prove_ms", "per_sec", "proof_len", "proof" (ark-serialize,
 * compressed)}; with reps > 1 the first prove (which builds the Lagrange basis and the MSM window
 * tables) is untimed and prove_ms is the mean of the other reps - 1.  Exit status: 0 valid
 * proof, 2 rejected by the verifier, 3 no gfx950 device, 1 any other error. */
#define _POSIX_C_SOURCE 199309L  // clock_gettime
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "tns.h"

static int fail(const char *what, int rc) {
  fprintf(stderr, "prove: %s failed (status %d): %s\n", what, rc, tns_last_error());
  return rc == TNS_ERR_NO_DEVICE ? 3 : 1;
}

static double now_ms(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e3 + t.tv_nsec / 1e6;
}

static size_t arg_size(int argc, char **argv, int i, size_t dflt) {
  return argc > i ? (size_t)strtoull(argv[i], NULL, 10) : dflt;
}

int main(int argc, char **argv) {
  const int shout = argc > 1 && strcmp(argv[1], "shout") == 0;
  if (argc < 2 || (!shout && strcmp(argv[1], "twist") != 0)) {
    fprintf(stderr, "usage: prove twist|shout [log_size [n [m [reps]]]]\n");
    return 1;
  }
  const unsigned log_size = (unsigned)arg_size(argc, argv, 2, 8);
  const size_t n = arg_size(argc, argv, 3, 256);  // operations (twist) / table entries (shout)
  const size_t m = arg_size(argc, argv, 4, shout ? 256 : (size_t)1 << log_size);  // memory size / lookups
  const int reps = (int)arg_size(argc, argv, 5, 1);
  const size_t units = shout ? m : n;  // what a second of proving is counted in

  tns_ctx *ctx = NULL;
  int rc = tns_ctx_create(0, &ctx);
  if (rc) return fail("tns_ctx_create", rc);
  int status = 1;
  tns_params pp;
  tns_srs *srs = NULL;
  const size_t na = (n ? n : 1), nb = (m ? m : 1);
  uint64_t *ints = malloc(sizeof(uint64_t) * na);    // addresses / table values as integers
  uint64_t *vals = malloc(sizeof(uint64_t) * na);    // trace values as integers (twist)
  uint64_t *fr = malloc(sizeof(uint64_t) * 4 * na);  // values / entries in Montgomery form
  uint64_t *idx = malloc(sizeof(uint64_t) * nb);     // lookup indices (shout)
  uint8_t *isw = malloc(na);
  tns_proof *proof = malloc(sizeof(tns_proof));
  uint8_t *bytes = NULL;
  if (!ints || !vals || !fr || !idx || !isw || !proof) {
    fprintf(stderr, "prove: host allocation failed\n");
    goto done;
  }
  if ((rc = tns_setup_params(ctx, log_size, &pp, &srs))) {
    status = fail("tns_setup_params", rc);
    goto done;
  }
  if (shout) {
    for (size_t i = 0; i < n; i++) ints[i] = (uint64_t)i * i;
    for (size_t j = 0; j < m; j++) idx[j] = n ? j % n : 0;
    tns_fr_from_u64(ints, n, fr);  // FieldElement::from(u64)
  } else {
    if ((rc = tns_bench_trace(m, n, ints, vals, isw))) {
      status = fail("tns_bench_trace", rc);
      goto done;
    }
    tns_fr_from_u64(vals, n, fr);
  }

  double t0 = now_ms();
  for (int r = 0; r < (reps > 1 ? reps : 1); r++) {
    if (r == 1) t0 = now_ms();  // the first of several proves is the warm-up
    rc = shout ? tns_shout_prove(ctx, srs, &pp, fr, n, idx, m, proof)
               : tns_twist_prove(ctx, srs, &pp, ints, fr, isw, n, proof);
    if (rc) {
      status = fail(shout ? "tns_shout_prove" : "tns_twist_prove", rc);
      goto done;
    }
  }
  const double ms = (now_ms() - t0) / (reps > 1 ? reps - 1 : 1);

  tns_vk vk;
  int ok = 0;
  if ((rc = tns_verifier_key(&pp, &vk)) ||
      (rc = shout ? tns_shout_verify(&vk, proof, &ok) : tns_twist_verify(&vk, proof, &ok))) {
    status = fail("verify", rc);
    goto done;
  }
  size_t len = 0;
  if ((rc = tns_proof_serialize(proof, 1, NULL, 0, &len))) {
    status = fail("tns_proof_serialize", rc);
    goto done;
  }
  bytes = malloc(len ? len : 1);
  if (!bytes || (rc = tns_proof_serialize(proof, 1, bytes, len, &len))) {
    status = bytes ? fail("tns_proof_serialize", rc) : 1;
    goto done;
  }
  printf("{\"ok\": %d, \"protocol\": \"%s\", \"log_size\": %u, \"n\": %zu, \"m\": %zu, \"prove_ms\": %.3f, "
         "\"per_sec\": %.1f, \"proof_len\": %zu, \"proof\": \"",
         ok, shout ? "shout" : "twist", log_size, n, m, ms, ms > 0 ? units / (ms / 1e3) : 0.0, len);
  for (size_t i = 0; i < len; i++) printf("%02x", bytes[i]);
  printf("\"}\n");
  status = ok ? 0 : 2;

done:
  free(bytes);
  free(proof);
  free(isw);
  free(idx);
  free(fr);
  free(vals);
  free(ints);
  if (srs) tns_srs_destroy(srs);
  tns_ctx_destroy(ctx);
  return status;
}
