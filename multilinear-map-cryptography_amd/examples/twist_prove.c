/* twist_prove.c -- a plain C host of the drop-in boundary (include/tns.h), no Python, no torch:
 * the calls a Rust binding of Twist::prove makes.
 *
 *   twist_prove [log_size [n_ops [memory_size [reps]]]]      defaults 8 256 2^log_size 1
 *
 * setup_params(log_size) (src/utils.rs:79-131), the ProtocolBenchmarks trace of n_ops operations
 * (src/benchmarks.rs:88-99), Twist::prove on host buffers (src/twist.rs:107-252, PCIe included),
 * Twist::verify (src/twist.rs:255-304), and the proof's ark-serialize bytes.  Prints one JSON
 * line {"ok", "prove_ms", "ops_per_sec", "proof_len", "proof"}; with reps > 1 the first prove
 * (which builds the Lagrange basis and the MSM window tables) is untimed and prove_ms is the
 * mean of the other reps - 1.  Exit status: 0 valid proof,
 * 2 rejected by the verifier, 3 no gfx950 device, 1 any other error. */
#define _POSIX_C_SOURCE 199309L  // clock_gettime
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "tns.h"

static int fail(const char *what, int rc) {
  fprintf(stderr, "twist_prove: %s failed (status %d): %s\n", what, rc, tns_last_error());
  return rc == TNS_ERR_NO_DEVICE ? 3 : 1;
}

static double now_ms(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e3 + t.tv_nsec / 1e6;
}

int main(int argc, char **argv) {
  const unsigned log_size = argc > 1 ? (unsigned)strtoul(argv[1], NULL, 10) : 8;
  const size_t n_ops = argc > 2 ? (size_t)strtoull(argv[2], NULL, 10) : 256;
  const size_t memory_size = argc > 3 ? (size_t)strtoull(argv[3], NULL, 10) : (size_t)1 << log_size;
  const int reps = argc > 4 ? atoi(argv[4]) : 1;

  tns_ctx *ctx = NULL;
  int rc = tns_ctx_create(0, &ctx);
  if (rc) return fail("tns_ctx_create", rc);
  int status = 1;
  tns_params pp;
  tns_srs *srs = NULL;
  uint64_t *addr = malloc(sizeof(uint64_t) * (n_ops ? n_ops : 1));
  uint64_t *val64 = malloc(sizeof(uint64_t) * (n_ops ? n_ops : 1));
  uint64_t *val = malloc(sizeof(uint64_t) * 4 * (n_ops ? n_ops : 1));
  uint8_t *isw = malloc(n_ops ? n_ops : 1);
  tns_proof *proof = malloc(sizeof(tns_proof));
  uint8_t *bytes = NULL;
  if (!addr || !val64 || !val || !isw || !proof) {
    fprintf(stderr, "twist_prove: host allocation failed\n");
    goto done;
  }
  if ((rc = tns_setup_params(ctx, log_size, &pp, &srs))) {
    status = fail("tns_setup_params", rc);
    goto done;
  }
  if ((rc = tns_bench_trace(memory_size, n_ops, addr, val64, isw))) {
    status = fail("tns_bench_trace", rc);
    goto done;
  }
  tns_fr_from_u64(val64, n_ops, val);  // FieldElement::from(u64), Montgomery limbs

  double t0 = now_ms();
  for (int r = 0; r < (reps > 1 ? reps : 1); r++) {
    if (r == 1) t0 = now_ms();  // the first of several proves is the warm-up
    if ((rc = tns_twist_prove(ctx, srs, &pp, addr, val, isw, n_ops, proof))) {
      status = fail("tns_twist_prove", rc);
      goto done;
    }
  }
  const double ms = (now_ms() - t0) / (reps > 1 ? reps - 1 : 1);

  tns_vk vk;
  int ok = 0;
  if ((rc = tns_verifier_key(&pp, &vk)) || (rc = tns_twist_verify(&vk, proof, &ok))) {
    status = fail("tns_twist_verify", rc);
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
  printf("{\"ok\": %d, \"log_size\": %u, \"n_ops\": %zu, \"prove_ms\": %.3f, \"ops_per_sec\": %.1f, "
         "\"proof_len\": %zu, \"proof\": \"",
         ok, log_size, n_ops, ms, ms > 0 ? n_ops / (ms / 1e3) : 0.0, len);
  for (size_t i = 0; i < len; i++) printf("%02x", bytes[i]);
  printf("\"}\n");
  status = ok ? 0 : 2;

done:
  free(bytes);
  free(proof);
  free(isw);
  free(val);
  free(val64);
  free(addr);
  if (srs) tns_srs_destroy(srs);
  tns_ctx_destroy(ctx);
  return status;
}
