/*
 * Host-side sanitizer driver for libdrandhip (test infrastructure): the library's host code (argument checks, scheme
 * registry, host SHA-256 DigestBeacon, error reporting, the no-device path of the worker pool, dh_shutdown) built
 * with -fsanitize=address,undefined and driven through the C ABI with no GPU present. Digests are compared with the
 * oracle's (crypto/schemes.go:106-114, 147-151). Exit 0 = all checks passed, no sanitizer report.
 */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/drandhip.h"

void or_digest_beacon(uint8_t *out, int sch, uint64_t round, const uint8_t *prev, size_t prevlen);

static int fails = 0;
#define CHECK(c, what)                    \
  do {                                    \
    if (!(c)) {                           \
      fprintf(stderr, "FAIL %s\n", what); \
      fails++;                            \
    }                                     \
  } while (0)

int main(void) {
  CHECK(dh_scheme_from_name("pedersen-bls-chained") == DH_SCHEME_CHAINED, "scheme id");
  CHECK(dh_scheme_from_name("bls-unchained-g1-rfc9380") == DH_SCHEME_G1_RFC9380, "quicknet id");
  CHECK(dh_scheme_from_name("nope") == DH_EINVAL && strstr(dh_last_error_string(), "nope"), "bad scheme");
  CHECK(dh_scheme_from_name(NULL) == DH_EINVAL, "null scheme");
  CHECK(dh_sig_len(0) == 96 && dh_key_len(3) == 96 && dh_sig_len(9) == DH_EINVAL, "lengths");
  /* DigestBeacon on the host for previous signatures of many lengths, against the oracle */
  uint8_t prevs[8][200], out[8 * 32], want[32];
  uint32_t lens[8] = {0, 1, 31, 32, 95, 96, 97, 200};
  uint64_t rounds[8];
  for (int i = 0; i < 8; i++) {
    rounds[i] = 1000u + (uint64_t)i * 77u;
    for (int k = 0; k < 200; k++) prevs[i][k] = (uint8_t)(i * 31 + k * 7);
  }
  CHECK(dh_digest_batch(DH_SCHEME_CHAINED, rounds, &prevs[0][0], 200, lens, 8, out) == DH_OK, "digest batch");
  for (int i = 0; i < 8; i++) {
    or_digest_beacon(want, 0, rounds[i], prevs[i], lens[i]);
    CHECK(memcmp(out + 32 * i, want, 32) == 0, "chained digest");
  }
  lens[3] = 201;
  CHECK(dh_digest_batch(DH_SCHEME_CHAINED, rounds, &prevs[0][0], 200, lens, 8, out) == DH_EINVAL, "length > stride");
  CHECK(dh_digest_batch(DH_SCHEME_UNCHAINED, rounds, NULL, 0, NULL, 8, out) == DH_OK, "unchained digest");
  or_digest_beacon(want, 1, rounds[5], NULL, 0);
  CHECK(memcmp(out + 32 * 5, want, 32) == 0, "unchained digest value");
  /* argument validation before any device work */
  uint8_t pk[96] = {0}, sig[96] = {0}, v[4];
  CHECK(dh_verify_batch(7, pk, 96, rounds, sig, 96, NULL, 0, NULL, 1, v, NULL, 0) == DH_EINVAL, "bad scheme id");
  CHECK(dh_verify_batch(3, NULL, 96, rounds, sig, 48, NULL, 0, NULL, 1, v, NULL, 0) == DH_EINVAL, "null key");
  CHECK(dh_verify_batch(0, pk, 48, rounds, sig, 96, &prevs[0][0], 32, lens + 4, 2, v, NULL, 0) == DH_EINVAL, "prev > stride");
  CHECK(dh_recover_batch(1, pk, 0, 3, NULL, NULL, NULL, 0, NULL, NULL) == DH_EINVAL, "t = 0");
  CHECK(dh_hash_to_curve(3, NULL, NULL, 0, (const uint8_t *)"x", 1, NULL) == DH_EINVAL, "bad group");
  CHECK(dh_init(3) == DH_EINVAL, "two devices in one mask");
  CHECK(dh_set_split(0, 0) == DH_EINVAL && dh_set_split(1024, 2) == DH_OK, "split");
  /* no GPU here: the pool reports a device error, cleanly */
  int rc = dh_verify_batch(3, pk, 96, rounds, sig, 48, NULL, 0, NULL, 1, v, NULL, 0);
  CHECK(rc == DH_EDEVICE || rc == DH_EKEY, "no-device path");
  char buf[64];
  CHECK(dh_profile(1) == DH_OK && dh_profile_read(buf, sizeof buf) >= 2 && dh_profile(0) == DH_OK, "profiler");
  dh_shutdown();
  dh_shutdown();
  if (fails) return 1;
  printf("libdrandhip host sanitizer driver: all checks passed\n");
  return 0;
}
