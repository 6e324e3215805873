/* A C client of libhipbls.so: what the cgo shim of INTEGRATION.md does, without Python.
 * Built by charon_amd/build.py (gcc -std=c99 -Wall -Wextra -Werror against include/hipbls.h), run
 * by tests/test_gpu_parity.py test_c_client with the reference's teku vector
 * (eth2util/signing/signing_test.go, tests/golden/kat_reference.json) on the command line:
 *   cabi_client <sk hex> <signing root hex> <teku signature hex>
 * It signs, derives the public key, verifies the teku signature and a corrupted copy, splits the
 * key 3-of-4, signs with the shares and threshold-aggregates them, and prints one JSON object. */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/hipbls.h"

static int unhex(const char* s, uint8_t* out, size_t n) {
  if (strlen(s) != 2 * n) return -1;
  for (size_t i = 0; i < n; i++) {
    unsigned v;
    if (sscanf(s + 2 * i, "%2x", &v) != 1) return -1;
    out[i] = (uint8_t)v;
  }
  return 0;
}

static void hex(const uint8_t* b, size_t n, char* out) {
  for (size_t i = 0; i < n; i++) sprintf(out + 2 * i, "%02x", b[i]);
}

int main(int argc, char** argv) {
  uint8_t sk[32], msg[32], teku[96];
  if (argc != 4 || unhex(argv[1], sk, 32) || unhex(argv[2], msg, 32) || unhex(argv[3], teku, 96)) {
    fprintf(stderr, "usage: cabi_client <sk hex> <root hex> <signature hex>\n");
    return 2;
  }
  if (hbls_init(0) != 0) {
    fprintf(stderr, "hbls_init: %s\n", hbls_last_error());
    return 1;
  }
  uint64_t off = 0;
  uint32_t len = 32;
  uint8_t sig[96], pk[48], st[8];
  if (hbls_sign_batch(sk, msg, &off, &len, 1, sig, st) || st[0] != HBLS_OK) return 1;
  if (hbls_secret_to_public_key_batch(sk, 1, pk, st) || st[0] != HBLS_OK) return 1;
  /* the teku signature, then the same with its last byte changed */
  uint8_t sigs[2 * 96], pks[2 * 48], msgs[2 * 32];
  uint64_t offs[2] = {0, 32};
  uint32_t lens[2] = {32, 32};
  memcpy(sigs, teku, 96);
  memcpy(sigs + 96, teku, 96);
  sigs[191] ^= 1;
  memcpy(pks, pk, 48);
  memcpy(pks + 48, pk, 48);
  memcpy(msgs, msg, 32);
  memcpy(msgs + 32, msg, 32);
  uint8_t vst[2] = {255, 255};
  if (hbls_verify_batch(pks, sigs, msgs, offs, lens, 2, vst)) return 1;
  int64_t first = -2;
  uint8_t fst = 255;
  if (hbls_verify_batch_first_error(pks, sigs, msgs, offs, lens, 2, &first, &fst, NULL)) return 1;
  /* 3-of-4 split of the key, three shares sign, ThresholdAggregate = the key's own signature */
  uint8_t coeffs[2 * 32] = {0}, shares[4 * 32], sst = 255;
  coeffs[31] = 7;
  coeffs[63] = 11;
  if (hbls_threshold_split(sk, coeffs, 4, 3, shares, &sst) || sst != HBLS_OK) return 1;
  uint8_t psig[3 * 96], pmsg[3 * 32];
  uint64_t poff[3] = {0, 32, 64};
  uint32_t plen[3] = {32, 32, 32};
  for (int k = 0; k < 3; k++) memcpy(pmsg + 32 * k, msg, 32);
  /* shares 2, 3, 4 (a non-prefix set) */
  if (hbls_sign_batch(shares + 32, pmsg, poff, plen, 3, psig, st) || st[0] || st[1] || st[2]) return 1;
  int64_t idx[3] = {2, 3, 4};  /* share i is f(i) */
  uint32_t goff[2] = {0, 3};
  uint8_t agg[96], ast = 255;
  if (hbls_threshold_aggregate_batch(psig, idx, goff, 1, agg, &ast)) return 1;
  char sh[193], ah[193];
  hex(sig, 96, sh);
  hex(agg, 96, ah);
  printf("{\"build\": \"%s\", \"sign_equals_teku\": %s, \"verify\": [%d, %d], \"first_error\": [%lld, %d], "
         "\"aggregate_status\": %d, \"aggregate_equals_signature\": %s, \"signature\": \"%s\", \"aggregate\": \"%s\"}\n",
         hbls_build_id(), memcmp(sig, teku, 96) == 0 ? "true" : "false", vst[0], vst[1], (long long)first, fst, ast,
         memcmp(agg, sig, 96) == 0 ? "true" : "false", sh, ah);
  return 0;
}
