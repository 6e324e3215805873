// Per-item building blocks shared by the gfx950 kernels (hipbls.hip):
// ZCash point (de)serialisation (herumi ETH mode, tbls/herumi.go:288-304 Deserialize/Serialize),
// and the Verify core e(pk, H(m)) * e(-g1, sig) == 1 (herumi.go:299 VerifyByte).
#pragma once
#include "h2c.h"
#include "pairing.h"
#include "fr.h"
#include "ec28.h"

namespace hb {

// status codes (include/hipbls.h)
enum : uint8_t {
  ST_OK = 0,
  ST_BAD_PUBKEY = 1,     // "cannot set compressed public key in Herumi format"
  ST_BAD_SIGNATURE = 2,  // "cannot unmarshal signature into Herumi signature"
  ST_NOT_VERIFIED = 3,   // "signature not verified" / "signature verification failed"
  ST_COMBINE_FAILED = 4, // "cannot combine signatures"
  ST_BAD_SECRET = 5,     // "cannot unmarshal secret into Herumi secret key"
  ST_BAD_INPUT = 6,      // malformed batch description (offsets / lengths)
  ST_UNCHECKED = 7,      // first-error mode: not decided (after the first failing item)
};

// Parse the 3 flag bits of a compressed encoding.  Returns false for an invalid combination;
// sets inf for the canonical infinity encoding 0xc0 || 0...
HD bool parse_flags(const uint8_t* b, int len, bool& inf, bool& sign) {
  uint8_t b0 = b[0];
  if (!(b0 & 0x80)) return false;  // uncompressed form is not accepted for 48/96-byte inputs
  inf = (b0 & 0x40) != 0;
  sign = (b0 & 0x20) != 0;
  if (inf) {
    if (sign) return false;
    uint32_t acc = b0 & 0x1f;
    for (int i = 1; i < len; i++) acc |= b[i];
    return acc == 0;
  }
  return true;
}

HDNI uint8_t g1_decompress(G1A& out, const uint8_t* b, bool subgroup_check = true) {
  bool inf, sign;
  if (!parse_flags(b, 48, inf, sign)) return 1;
  if (inf) {
    out.x = fp_zero();
    out.y = fp_zero();
    out.inf = true;
    return 0;
  }
  uint8_t tmp[48];
  for (int i = 0; i < 48; i++) tmp[i] = b[i];
  tmp[0] &= 0x1f;
  Fp xr;
  fp_from_be_raw(xr, tmp);
  if (!fp_raw_lt_p(xr)) return 1;
  Fp x = fp_to_mont(xr);
  Fp y2 = fp_add(fp_mul(fp_sqr(x), x), fp_from_const(G1_B));
  Fp y;
  if (!fp_sqrt(y, y2)) return 1;
  if (fp_raw_is_lex_largest(fp_from_mont(y)) != sign) y = fp_neg(y);
  out.x = x;
  out.y = y;
  out.inf = false;
  if (subgroup_check && !g1_in_subgroup28(out)) return 1;
  return 0;
}

HDNI uint8_t g2_decompress(G2A& out, const uint8_t* b, bool subgroup_check = true) {
  bool inf, sign;
  if (!parse_flags(b, 96, inf, sign)) return 1;
  if (inf) {
    out.x = f2_zero();
    out.y = f2_zero();
    out.inf = true;
    return 0;
  }
  uint8_t tmp[48];
  for (int i = 0; i < 48; i++) tmp[i] = b[i];
  tmp[0] &= 0x1f;
  Fp x1r, x0r;
  fp_from_be_raw(x1r, tmp);
  fp_from_be_raw(x0r, b + 48);
  if (!fp_raw_lt_p(x1r) || !fp_raw_lt_p(x0r)) return 1;
  Fp2 x = {fp_to_mont(x0r), fp_to_mont(x1r)};
  Fp2 y2 = f2_add(f2_mul(f2_sqr(x), x), f2_from_const(G2_B));
  Fp2 y;
  if (!f2_sqrt(y, y2)) return 1;
  if (f2_is_lex_largest(y) != sign) y = f2_neg(y);
  out.x = x;
  out.y = y;
  out.inf = false;
  if (subgroup_check && !g2_in_subgroup28(out)) return 1;
  return 0;
}

HDNI void g1_compress(uint8_t* b, const G1A& p) {
  if (p.inf) {
    b[0] = 0xc0;
    for (int i = 1; i < 48; i++) b[i] = 0;
    return;
  }
  fp_to_be_raw(b, fp_from_mont(p.x));
  b[0] |= 0x80;
  if (fp_raw_is_lex_largest(fp_from_mont(p.y))) b[0] |= 0x20;
}

HDNI void g2_compress(uint8_t* b, const G2A& p) {
  if (p.inf) {
    b[0] = 0xc0;
    for (int i = 1; i < 96; i++) b[i] = 0;
    return;
  }
  fp_to_be_raw(b, fp_from_mont(p.x.c1));
  fp_to_be_raw(b + 48, fp_from_mont(p.x.c0));
  b[0] |= 0x80;
  if (f2_is_lex_largest(p.y)) b[0] |= 0x20;
}

HD G1A g1_generator_neg() {
  return {fp_from_const(G1_GEN_X), fp_from_const(G1_GEN_NEG_Y), false};
}

HD G1A g1_generator() { return {fp_from_const(G1_GEN_X), fp_from_const(G1_GEN_Y), false}; }

// e(pk, hm) * e(-g1, sig) == 1 ?   pk, hm, sig already validated (on curve, in subgroup).
HDNI bool verify_core(const G1A& pk, const G2A& hm, const G2A& sig) {
  if (pk.inf) return false;  // KeyValidate: identity public key never verifies
  if (sig.inf) return false;  // e(pk, H(m)) != 1 for pk != O, H(m) != O
  if (hm.inf) return false;
  Fp12 f = miller_loop2(pk, hm, g1_generator_neg(), sig);
  return f12_is_one(final_exponentiation(f));
}

}  // namespace hb
