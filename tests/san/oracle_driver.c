/*
 * Sanitizer driver (test infrastructure): the CPU oracle built with -fsanitize=address,undefined and run over the
 * reference's known-answer tests (/root/reference/crypto/schemes_test.go:90-115, crypto/curve_test.go:12-20), the
 * RFC 9380 K.1 expand_message_xmd vectors, a sign / verify round trip per scheme, malformed encodings and a small
 * tbls Recover. Exit status 0 = every check passed and no sanitizer report (the sanitizers abort on error).
 */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

int or_verify_beacon(int sch, const uint8_t *pk, size_t pklen, uint64_t round, const uint8_t *sig, size_t siglen,
                     const uint8_t *prev, size_t prevlen);
int or_sign(int sch, const uint8_t *sk32, const uint8_t *msg, size_t mlen, uint8_t *sig_out);
int or_public_key(int sch, const uint8_t *sk32, uint8_t *pk_out);
void or_digest_beacon(uint8_t *out, int sch, uint64_t round, const uint8_t *prev, size_t prevlen);
void or_expand_message_xmd(uint8_t *out, size_t len, const uint8_t *msg, size_t mlen, const uint8_t *dst, size_t dlen);
int or_decode(int g2, const uint8_t *b);
int or_recover(int sch, const uint8_t *commits, int t, int n, const uint8_t *msg, size_t mlen, const uint8_t *partials,
               int npart, uint8_t *sig_out);
void or_init(int fast_subgroup);

static int hexdec(uint8_t *out, const char *h) {
  size_t n = strlen(h) / 2;
  for (size_t i = 0; i < n; i++) {
    unsigned v;
    sscanf(h + 2 * i, "%2x", &v);
    out[i] = (uint8_t)v;
  }
  return (int)n;
}

static int fails = 0;
#define CHECK(c, what)                   \
  do {                                   \
    if (!(c)) {                          \
      fprintf(stderr, "FAIL %s\n", what); \
      fails++;                           \
    }                                    \
  } while (0)

int main(void) {
  or_init(0);
  uint8_t pk[96], sig[96], prev[96];
  /* schemes_test.go:90-96 (chained, mainnet) */
  int pl = hexdec(pk, "868f005eb8e6e4ca0a47c8a77ceaa5309a47978a7c71bc5cce96366b5d7a569937c529eeda66c7293784a9402801af31");
  int sl = hexdec(sig, "814778ed1e480406beb43b74af71ce2f0373e0ea1bfdfea8f9ed62c876c20fcbc7f0163860e3da42ed2148756015f4551451898ffe06d384b4d002245025571b6b7a752f7158b40ad92b13b6d703ad31922a617f2c7f6d960b84d56cf1d79eef");
  int rl = hexdec(prev, "8bd96294383b4d1e04e736360bd7a487f9f409f1e7bd800b720656a310d577b3bdb1e1631af6c5782a1d8979c502f395036181eff4058960fc40bb7034cdae1991d3eda518ab204a077d2f7e724974cf87b407e549bd815cf0b8e5a3832f675d");
  CHECK(or_verify_beacon(0, pk, pl, 2634945, sig, sl, prev, rl) == 1, "chained KAT");
  CHECK(or_verify_beacon(0, pk, pl, 2634946, sig, sl, prev, rl) == 0, "chained KAT, wrong round");
  CHECK(or_verify_beacon(0, pk, pl, 2634945, sig, sl - 1, prev, rl) == 0, "chained KAT, short signature");
  CHECK(or_verify_beacon(0, pk, pl, 2634945, sig, sl, prev, 31) == 0, "chained KAT, 31-byte prev");
  /* schemes_test.go:110-115 (bls-unchained-on-g1) */
  pl = hexdec(pk, "876f6fa8073736e22f6ff4badaab35c637503718f7a452d178ce69c45d2d8129a54ad2f988ab10c9666f87ab603c59bf013409a5b500555da31720f8eec294d9809b8796f40d5372c71a44ca61226f1eb978310392f98074a608747f77e66c5a");
  sl = hexdec(sig, "ac7c3ca14bc88bd014260f22dc016b4fe586f9313c3a549c83d195811a99a5d2d4999d4df6daec73ff51fafadd6d5bb5");
  CHECK(or_verify_beacon(2, pk, pl, 3, sig, sl, NULL, 0) == 1, "g1 KAT");
  /* curve_test.go:12-20: fixed key + 18-byte message -> exact G2 signature */
  uint8_t sk[32], msg[18], want[96], got[96];
  hexdec(sk, "643d6c704505385387a20d98aba19664e3ee81c600d21a0da910cc87f5dc4ab3");
  hexdec(msg, "7061737320746865207369676e6174757265");
  hexdec(want, "9940ca447bab3bab393c3a07866349343630437167eaeab063ef1e47acedc51e85c513121cf319a8832c3d136d7f36490fa7241194b403a3bbbba9e7d5e73c9a86f67a9585c6fe077cd6576b2f76560efbab3550d9d5124242c728e3a7ef6989");
  or_sign(0, sk, msg, sizeof msg, got);
  CHECK(memcmp(got, want, 96) == 0, "sign KAT");
  /* RFC 9380 K.1 */
  uint8_t x[32], wx[32];
  const char *dst = "QUUX-V01-CS02-with-expander-SHA256-128";
  or_expand_message_xmd(x, 32, (const uint8_t *)"", 0, (const uint8_t *)dst, strlen(dst));
  hexdec(wx, "68a985b87eb6b46952128911f2a4412bbc302a9d759667f87f7a21d803f07235");
  CHECK(memcmp(x, wx, 32) == 0, "xmd K.1 empty");
  /* round trips and malformed encodings for every scheme */
  for (int s = 0; s < 4; s++) {
    uint8_t key[96], d[32], sg[96];
    const int g2sig = s < 2;
    or_public_key(s, sk, key);
    or_digest_beacon(d, s, 1234, s == 0 ? prev : NULL, s == 0 ? 96 : 0);
    or_sign(s, sk, d, 32, sg);
    CHECK(or_verify_beacon(s, key, g2sig ? 48 : 96, 1234, sg, g2sig ? 96 : 48, s == 0 ? prev : NULL, s == 0 ? 96 : 0) == 1,
          "round trip");
    sg[0] &= 0x7f; /* compression flag cleared */
    CHECK(or_decode(g2sig, sg) != 1, "uncompressed flag rejected");
    memset(sg, 0xff, 96);
    CHECK(or_decode(g2sig, sg) != 1, "x >= p rejected");
  }
  /* tbls: t = 2, n = 3 with the dealer polynomial f(x) = a0 + a1 x, shares f(i + 1) */
  {
    uint8_t a0[32] = {0}, a1[32] = {0}, s1[32] = {0}, s2[32] = {0}, commits[96], d[32], parts[2 * 98], rec[96], grp[96];
    a0[31] = 7; a1[31] = 5; s1[31] = 7 + 5 * 1; s2[31] = 7 + 5 * 3; /* shares of indices 0 and 2 */
    or_public_key(1, a0, commits);
    or_public_key(1, a1, commits + 48);
    or_digest_beacon(d, 1, 99, NULL, 0);
    parts[0] = 0; parts[1] = 0; or_sign(1, s1, d, 32, parts + 2);
    parts[98] = 0; parts[99] = 2; or_sign(1, s2, d, 32, parts + 100);
    CHECK(or_recover(1, commits, 2, 3, d, 32, parts, 2, rec) == 96, "recover status");
    or_sign(1, a0, d, 32, grp);
    CHECK(memcmp(rec, grp, 96) == 0, "recover = [f(0)] H(m)");
  }
  if (fails) return 1;
  printf("oracle sanitizer driver: all checks passed\n");
  return 0;
}
