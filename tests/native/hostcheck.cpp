// TEST-ONLY harness: compiles the kernels' per-item arithmetic (charon_amd/csrc/*.h) for the
// host CPU so tests/test_hostcheck.py can compare it with the Python oracle without a GPU.
// The product library (libhipbls.so) never loads this; it is not a fallback.
// Built with HB_COUNT_OPS: every Fp / Fr Montgomery product bumps a thread-local counter, which
// hc_count_* read to freeze the algorithmic work per item (charon_amd/opcounts.py).
#define HB_COUNT_OPS 1
#include "../../charon_amd/csrc/ops.h"
#include "../../charon_amd/csrc/rlc.h"
#include "../../charon_amd/csrc/ta_small.h"
#include "../../charon_amd/csrc/pair28.h"
#include <string.h>

namespace hb {
thread_local unsigned long long g_cnt_fp_mul = 0, g_cnt_fr_mul = 0;
}

// host restatement of lines.h line_chain (68 lines of the Miller chain of Q)
struct LineEntryHost {
  hb::Fp2 a0, a1, b1;
};
static void hc_line_chain(const hb::G2A& Q, LineEntryHost* out, bool eval) {
  using namespace hb;
  G2Proj T = {Q.x, Q.y, f2_one()};
  int j = 0;
  for (int i = 62; i >= 0; i--) {
    LineCoeffs l = miller_dbl_c(T);
    if (eval) line_eval(l, fp_from_const(G1_GEN_X), fp_from_const(G1_GEN_NEG_Y));
    out[j++] = {l.a0, l.a1, l.b1};
    if ((HB_X_ABS >> i) & 1) {
      l = miller_add_c(T, Q.x, Q.y);
      if (eval) line_eval(l, fp_from_const(G1_GEN_X), fp_from_const(G1_GEN_NEG_Y));
      out[j++] = {l.a0, l.a1, l.b1};
    }
  }
}

using namespace hb;

extern "C" {

// Fp-mul counts of the kernels' per-item stages, in the kernels' own call structure:
// out[0] k_verify (G1 decompress+subgroup, G2 decompress+subgroup, verify_core),
// out[1] k_hash_to_g2 (hash_to_g2 + affine conversion), out[2..4] the three k_verify stages.
// Returns the verify status.
int hc_count_verify(const uint8_t* pk48, const uint8_t* msg, uint32_t len, const uint8_t* sig96,
                    unsigned long long* out) {
  g_cnt_fp_mul = 0;
  G2A h = jac_to_aff(hash_to_g2(msg, len));
  out[1] = g_cnt_fp_mul;
  g_cnt_fp_mul = 0;
  G1A pk;
  G2A sig;
  int st = ST_OK;
  if (g1_decompress(pk, pk48)) st = ST_BAD_PUBKEY;
  out[2] = g_cnt_fp_mul;
  g_cnt_fp_mul = 0;
  if (!st && g2_decompress(sig, sig96)) st = ST_BAD_SIGNATURE;
  out[3] = g_cnt_fp_mul;
  g_cnt_fp_mul = 0;
  if (!st && !verify_core(pk, h, sig)) st = ST_NOT_VERIFIED;
  out[4] = g_cnt_fp_mul;
  out[0] = out[2] + out[3] + out[4];
  return st;
}

// k_group_member work for one partial of a ThresholdAggregate over k partials (index j):
// out[0] Fp-mul (decompress + subgroup + scalar multiplication), out[1] Fr-mul (lambda_j).
int hc_count_ta_member(const uint8_t* sigs, const int64_t* idx, int k, int j, unsigned long long* out) {
  g_cnt_fp_mul = 0;
  g_cnt_fr_mul = 0;
  G2A s;
  if (g2_decompress(s, sigs + 96 * j)) return ST_BAD_SIGNATURE;
  Fr xi = fr_from_i64(idx[j]);
  Fr num = fr_one(), den = fr_one();
  for (int m = 0; m < k; m++) {
    if (m == j) continue;
    Fr xm = fr_from_i64(idx[m]);
    num = fr_mul(num, xm);
    den = fr_mul(den, fr_sub(xm, xi));
  }
  Fr lam = fr_from_mont(fr_mul(num, fr_inv(den)));
  G2J p = jac_mul_aff(s, lam.v, 255);
  (void)p;
  out[0] = g_cnt_fp_mul;
  out[1] = g_cnt_fr_mul;
  return 0;
}

int hc_hash_to_g2(const uint8_t* msg, uint32_t len, uint8_t* out96) {
  G2J h = hash_to_g2(msg, len);
  g2_compress(out96, jac_to_aff(h));
  return 0;
}

int hc_g1_roundtrip(const uint8_t* in48, uint8_t* out48, int subgroup) {
  G1A p;
  uint8_t st = g1_decompress(p, in48, subgroup != 0);
  if (st) return st;
  g1_compress(out48, p);
  return 0;
}

int hc_g2_roundtrip(const uint8_t* in96, uint8_t* out96, int subgroup) {
  G2A p;
  uint8_t st = g2_decompress(p, in96, subgroup != 0);
  if (st) return st;
  g2_compress(out96, p);
  return 0;
}

int hc_sk_to_pk(const uint8_t* sk, uint8_t* out48) {
  Fr s;
  if (!fr_from_be(s, sk)) return ST_BAD_SECRET;
  G1J p = jac_mul_aff(g1_generator(), s.v, 256);
  g1_compress(out48, jac_to_aff(p));
  return 0;
}

int hc_sign(const uint8_t* sk, const uint8_t* msg, uint32_t len, uint8_t* out96) {
  Fr s;
  if (!fr_from_be(s, sk)) return ST_BAD_SECRET;
  G2A h = jac_to_aff(hash_to_g2(msg, len));
  G2J sig = jac_mul_aff(h, s.v, 256);
  g2_compress(out96, jac_to_aff(sig));
  return 0;
}

int hc_verify(const uint8_t* pk48, const uint8_t* msg, uint32_t len, const uint8_t* sig96) {
  G1A pk;
  if (g1_decompress(pk, pk48)) return ST_BAD_PUBKEY;
  G2A sig;
  if (g2_decompress(sig, sig96)) return ST_BAD_SIGNATURE;
  G2A h = jac_to_aff(hash_to_g2(msg, len));
  return verify_core(pk, h, sig) ? ST_OK : ST_NOT_VERIFIED;
}

// e(P, Q)^3 (our Miller function and final exponentiation), 12 Fp2 coefficients canonical BE
// in order c0.c0, c0.c1, c0.c2, c1.c0, c1.c1, c1.c2 (each c0 then c1 of the Fp2).
int hc_pairing(const uint8_t* pk48, const uint8_t* sig96, uint8_t* out576) {
  G1A p;
  G2A q;
  if (g1_decompress(p, pk48)) return 1;
  if (g2_decompress(q, sig96)) return 2;
  Fp12 f = final_exponentiation(miller_loop1(p, q));
  const Fp2* cs[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
  for (int i = 0; i < 6; i++) {
    fp_to_be_raw(out576 + 96 * i, fp_from_mont(cs[i]->c0));
    fp_to_be_raw(out576 + 96 * i + 48, fp_from_mont(cs[i]->c1));
  }
  return 0;
}

// Fp multiply of canonical big-endian values (sanity check of the Montgomery code)
int hc_fp_mul(const uint8_t* a48, const uint8_t* b48, uint8_t* out48) {
  Fp a, b;
  fp_from_be_raw(a, a48);
  fp_from_be_raw(b, b48);
  Fp r = fp_from_mont(fp_mul(fp_to_mont(a), fp_to_mont(b)));
  fp_to_be_raw(out48, r);
  return 0;
}

// Fp2 product and square of raw Montgomery-domain values (lazily reduced: anything below 2p), as the
// kernels hold them: a = (a0, a1), b = (b0, b1) as 48-byte big-endian numbers; out = a b / R and
// a^2 / R (R = 2^392), raw
int hc_fp2_mul_raw(const uint8_t* a96, const uint8_t* b96, uint8_t* out96, uint8_t* sq96) {
  Fp a0, a1, b0, b1, r0, r1;
  fp_from_be_raw(a0, a96);
  fp_from_be_raw(a1, a96 + 48);
  fp_from_be_raw(b0, b96);
  fp_from_be_raw(b1, b96 + 48);
  fp2_mul_core(r0.v, r1.v, a0.v, a1.v, b0.v, b1.v);
  fp_to_be_raw(out96, r0);
  fp_to_be_raw(out96 + 48, r1);
  fp2_sqr_core(r0.v, r1.v, a0.v, a1.v);
  fp_to_be_raw(sq96, r0);
  fp_to_be_raw(sq96 + 48, r1);
  return 0;
}

int hc_fp2_sqrt(const uint8_t* a96, uint8_t* out96) {
  Fp a0, a1;
  fp_from_be_raw(a0, a96);
  fp_from_be_raw(a1, a96 + 48);
  Fp2 a = {fp_to_mont(a0), fp_to_mont(a1)}, x;
  if (!f2_sqrt(x, a)) return 1;
  fp_to_be_raw(out96, fp_from_mont(x.c0));
  fp_to_be_raw(out96 + 48, fp_from_mont(x.c1));
  return 0;
}

int hc_lagrange_g2(const uint8_t* sigs, const int64_t* idx, int k, uint8_t* out96) {
  G2J acc = jac_infinity<Fp2>();
  for (int i = 0; i < k; i++) {
    G2A s;
    if (g2_decompress(s, sigs + 96 * i)) return ST_BAD_SIGNATURE;
    Fr xi = fr_from_i64(idx[i]);
    Fr num = fr_one(), den = fr_one();
    for (int j = 0; j < k; j++) {
      if (j == i) continue;
      Fr xj = fr_from_i64(idx[j]);
      num = fr_mul(num, xj);
      den = fr_mul(den, fr_sub(xj, xi));
    }
    if (fr_is_zero(den) || fr_is_zero(num)) return ST_COMBINE_FAILED;
    Fr lam = fr_from_mont(fr_mul(num, fr_inv(den)));
    acc = jac_add(acc, jac_mul_aff(s, lam.v, 256));
  }
  g2_compress(out96, jac_to_aff(acc));
  return 0;
}

}  // extern "C"

extern "C" {
static void put_fp2(uint8_t* o, const Fp2& a) {
  fp_to_be_raw(o, fp_from_mont(a.c0));
  fp_to_be_raw(o + 48, fp_from_mont(a.c1));
}
// stage dumps for debugging hash_to_g2: u0,u1 | sswu(u0) x,y | iso(sswu(u0)) affine x,y
int hc_h2c_stages(const uint8_t* msg, uint32_t len, uint8_t* out) {
  Fp2 u0, u1;
  hash_to_field_fp2(u0, u1, msg, len);
  put_fp2(out, u0);
  put_fp2(out + 96, u1);
  Fp2 x, y;
  sswu_map(x, y, u0);
  put_fp2(out + 192, x);
  put_fp2(out + 288, y);
  G2A q = jac_to_aff(iso3_map(x, y));
  put_fp2(out + 384, q.x);
  put_fp2(out + 480, q.y);
  return 0;
}
}
extern "C" {
static Fp2 get_fp2(const uint8_t* i) {
  Fp a, b;
  fp_from_be_raw(a, i);
  fp_from_be_raw(b, i + 48);
  return {fp_to_mont(a), fp_to_mont(b)};
}
// in: affine P (x,y) 192 bytes; out: psi(P) | [|x|]P | 2P | clear_cofactor(P) | P+psi(P)  (affine x,y each)
int hc_g2_debug(const uint8_t* in, uint8_t* out) {
  G2A p = {get_fp2(in), get_fp2(in + 96), false};
  G2J P = jac_from_aff(p);
  G2J outs[5] = {g2_psi(P), jac_mul_by_xabs(P), jac_dbl(P), g2_clear_cofactor(P), jac_add(P, g2_psi(P))};
  for (int i = 0; i < 5; i++) {
    G2A a = jac_to_aff(outs[i]);
    put_fp2(out + 192 * i, a.x);
    put_fp2(out + 192 * i + 96, a.y);
  }
  return 0;
}
}
extern "C" {
int hc_h2c_sum(const uint8_t* msg, uint32_t len, uint8_t* out) {
  Fp2 u0, u1;
  hash_to_field_fp2(u0, u1, msg, len);
  Fp2 x, y;
  sswu_map(x, y, u0);
  G2J q0 = iso3_map(x, y);
  sswu_map(x, y, u1);
  G2J q1 = iso3_map(x, y);
  G2J s = jac_add(q0, q1);
  G2A a = jac_to_aff(s);
  put_fp2(out, a.x); put_fp2(out + 96, a.y);
  G2A a0 = jac_to_aff(q1);
  put_fp2(out + 192, a0.x); put_fp2(out + 288, a0.y);
  G2A c = jac_to_aff(g2_clear_cofactor(s));
  put_fp2(out + 384, c.x); put_fp2(out + 480, c.y);
  return 0;
}
}

// CPU baseline for bench.py (reported, not the target): `units` validators of one slot, each =
// n partial Verifies (each hashing its message to G2, as herumi's VerifyByte does per call) + one
// ThresholdAggregate over shares 1..t, compared with the root-key signature.  std::thread workers
// take validators round-robin.  Returns the number of validators whose verdicts or aggregate
// differ from the expected (all valid, aggregate == root signature).
#include <atomic>
#include <thread>
#include <vector>
// build provenance (charon_amd/build.py hostcheck_build_id): the sources and flags this harness was
// compiled from; build_hostcheck reuses a harness only when the id matches the tree, and bench.py's
// cpu_baseline reports it
#ifndef HC_BUILD_ID
#define HC_BUILD_ID "hbls-hostcheck:(unstamped)"
#endif
extern "C" const char* hc_build_id() { return HC_BUILD_ID; }

extern "C" int hc_cpu_slot(int threads, int units, int n, int t, const uint8_t* pks, const uint8_t* sigs,
                           const uint8_t* msgs, const uint32_t* midx, const uint8_t* ta_sigs,
                           const uint8_t* root_sigs, const int64_t* ta_idx) {
  std::atomic<int> next{0}, bad{0};
  auto work = [&]() {
    for (;;) {
      int v = next.fetch_add(1);
      if (v >= units) return;
      bool ok = true;
      for (int i = v * n; i < v * n + n; i++)
        ok &= hc_verify(pks + 48ull * i, msgs + 32ull * midx[i], 32, sigs + 96ull * i) == 0;
      uint8_t out[96];
      ok &= hc_lagrange_g2(ta_sigs + 96ull * t * v, ta_idx + (size_t)t * v, t, out) == 0;
      ok &= memcmp(out, root_sigs + 96ull * v, 96) == 0;
      if (!ok) bad.fetch_add(1);
    }
  };
  std::vector<std::thread> ws;
  for (int k = 0; k < threads; k++) ws.emplace_back(work);
  for (auto& w : ws) w.join();
  return bad.load();
}

// ---------------------------------------------------------------------------------------
// Batched verification (vbatch.hip) on the host.
// hc_rlc: [a + b lambda] P and S through the endomorphism ladders of rlc.h, compressed
// (out48, out96); tests/test_hostcheck.py compares them with the oracle's [r] P, [r] S.
extern "C" int hc_rlc(const uint8_t* pk48, const uint8_t* sig96, uint32_t a, uint32_t b, uint8_t* out48,
                      uint8_t* out96) {
  G1A p;
  G2A q;
  if (g1_decompress(p, pk48)) return 1;
  if (g2_decompress(q, sig96)) return 2;
  g1_compress(out48, jac_to_aff(rlc_g1(p, a, b)));
  g2_compress(out96, jac_to_aff(rlc_g2(q, a, b)));
  return 0;
}

// Fp-mul counts of the building blocks the per-kernel roofline counts are assembled from
// (charon_amd/opcounts.py), on a valid (pk, sig):
//  0 f12_sqr            1 f12_mul_line        2 final_exponentiation   3 fp_inv
//  4 g1_decompress      5 g2_decompress       6 rlc_g1 (a, b top bits set)  7 rlc_g2
//  8 jac_add G1         9 jac_add G2          10 jac_to_aff G1 (Z != 1)     11 jac_to_aff G2
//  12 line chain at -g1 (68 lines, evaluated) 13 line chain unevaluated     14 jac_dbl G2
//  15 jac_add_aff G2    16 f12_cyclo_sqr      17 f12_mul                    18 g2_compress
extern "C" int hc_count_blocks(const uint8_t* pk48, const uint8_t* sig96, unsigned long long* out) {
  G1A p;
  G2A q;
  if (g1_decompress(p, pk48)) return 1;
  if (g2_decompress(q, sig96)) return 2;
  Fp12 f = miller_loop2(p, q, g1_generator_neg(), q);
  auto cnt = [&](int k, auto&& fn) {
    g_cnt_fp_mul = 0;
    fn();
    out[k] = g_cnt_fp_mul;
  };
  Fp12 r;
  cnt(0, [&] { r = f12_sqr(f); });
  cnt(1, [&] { r = f12_mul_line(f, q.x, q.y, q.x); });
  cnt(2, [&] { r = final_exponentiation(f); });
  Fp t;
  cnt(3, [&] { t = fp_inv(p.x); });
  G1A p2;
  G2A q2;
  cnt(4, [&] { g1_decompress(p2, pk48); });
  cnt(5, [&] { g2_decompress(q2, sig96); });
  G1J pj;
  G2J qj;
  cnt(6, [&] { pj = rlc_g1(p, 0x80000001u, 0x80000001u); });
  cnt(7, [&] { qj = rlc_g2(q, 0x80000001u, 0x80000001u); });
  G1J pj2 = jac_dbl(pj);
  G2J qj2 = jac_dbl(qj);
  cnt(8, [&] { pj2 = jac_add(pj2, pj); });
  cnt(9, [&] { qj2 = jac_add(qj2, qj); });
  cnt(10, [&] { p2 = jac_to_aff(pj2); });
  cnt(11, [&] { q2 = jac_to_aff(qj2); });
  static LineEntryHost lines[N_LINES];
  cnt(12, [&] { hc_line_chain(q, lines, true); });
  cnt(13, [&] { hc_line_chain(q, lines, false); });
  cnt(14, [&] { qj2 = jac_dbl(qj2); });
  cnt(15, [&] { qj2 = jac_add_aff(qj2, q); });
  Fp12 fe = final_exponentiation(f);
  cnt(16, [&] { r = f12_cyclo_sqr(fe); });
  cnt(17, [&] { r = f12_mul(f, fe); });
  uint8_t buf[96];
  cnt(18, [&] { g2_compress(buf, q); });
  cnt(19, [&] { pj2 = jac_add_aff(pj2, p); });
  cnt(20, [&] { pj2 = jac_dbl(pj2); });
  (void)r;
  (void)t;
  return 0;
}

// The batched verification's group check on the host (vbatch.hip k_rlc + k_group_prep + the
// pairing product): k items over one message with coefficients (a_i, b_i).  Returns 1 if the
// combined equation holds, 0 if not, <0 on a decoding error.
extern "C" int hc_group_check(int k, const uint8_t* pks, const uint8_t* sigs, const uint8_t* msg, uint32_t len,
                              const uint32_t* a, const uint32_t* b) {
  G1J pacc = jac_infinity<Fp>();
  G2J sacc = jac_infinity<Fp2>();
  for (int i = 0; i < k; i++) {
    G1A p;
    G2A q;
    if (g1_decompress(p, pks + 48 * i)) return -1;
    if (g2_decompress(q, sigs + 96 * i)) return -2;
    pacc = jac_add(pacc, rlc_g1(p, a[i], b[i]));
    sacc = jac_add(sacc, rlc_g2(q, a[i], b[i]));
  }
  G1A P = jac_to_aff(pacc);
  G2A S = jac_to_aff(sacc);
  G2A H = jac_to_aff(hash_to_g2(msg, len));
  Fp12 f = miller_loop2(P, H, g1_generator_neg(), S);
  return f12_is_one(final_exponentiation(f)) ? 1 : 0;
}

// Raw device Jacobian points (G1JEntry / G2JEntry limbs) -> compressed affine encodings.
extern "C" int hc_jac_compress(const uint8_t* g1raw, uint8_t* out48, const uint8_t* g2raw, uint8_t* out96) {
  G1J p;
  G2J q;
  memcpy(&p, g1raw, sizeof(p));
  memcpy(&q, g2raw, sizeof(q));
  g1_compress(out48, jac_to_aff(p));
  g2_compress(out96, jac_to_aff(q));
  return 0;
}

// The batched verification's coefficients on the host (vbatch.hip rlc_coeffs).
extern "C" void hc_rlc_coeffs(const uint32_t* key8, uint32_t item, uint32_t* ab) {
  uint32_t w[16];
  for (int j = 0; j < 8; j++) w[j] = key8[j];
  w[8] = item;
  w[9] = 0x80000000u;
  for (int j = 10; j < 15; j++) w[j] = 0;
  w[15] = 36 * 8;
  Sha256State st = sha256_init();
  sha256_compress(st, w);
  ab[0] = st.h[0];
  ab[1] = st.h[1];
  if ((ab[0] | ab[1]) == 0) ab[0] = 1;
}

// G1AEntry-layout affine point (x, y Montgomery limbs, inf) -> compressed
extern "C" int hc_g1a_compress(const uint8_t* raw, uint8_t* out48) {
  G1A p;
  memcpy(&p.x, raw, sizeof(Fp));
  memcpy(&p.y, raw + sizeof(Fp), sizeof(Fp));
  uint32_t inf;
  memcpy(&inf, raw + 2 * sizeof(Fp), 4);
  p.inf = inf != 0;
  g1_compress(out48, p);
  return 0;
}

// sum over k items of [a_i + b_i lambda] pk_i (G1), compressed
extern "C" int hc_rlc_sum_g1(int k, const uint8_t* pks, const uint32_t* ab, uint8_t* out48) {
  G1J acc = jac_infinity<Fp>();
  for (int i = 0; i < k; i++) {
    G1A p;
    if (g1_decompress(p, pks + 48 * i)) return 1;
    acc = jac_add(acc, rlc_g1(p, ab[2 * i], ab[2 * i + 1]));
  }
  g1_compress(out48, jac_to_aff(acc));
  return 0;
}

extern "C" int hc_jac_add(const uint8_t* pk48, const uint8_t* sig96, uint32_t k1, uint32_t k2, uint8_t* out48,
                          uint8_t* out96) {
  G1A p;
  G2A q;
  if (g1_decompress(p, pk48) || g2_decompress(q, sig96)) return 1;
  g1_compress(out48, jac_to_aff(jac_add(jac_mul_aff(p, &k1, 32), jac_mul_aff(p, &k2, 32))));
  g2_compress(out96, jac_to_aff(jac_add(jac_mul_aff(q, &k1, 32), jac_mul_aff(q, &k2, 32))));
  return 0;
}

extern "C" int hc_sum_raw(const uint8_t* pr_raw, uint32_t n, uint8_t* out48) {
  G1J acc = jac_infinity<Fp>();
  for (uint32_t i = 0; i < n; i++) {
    G1J p;
    memcpy(&p, pr_raw + sizeof(G1J) * i, sizeof(G1J));
    acc = jac_add(acc, p);
  }
  g1_compress(out48, jac_to_aff(acc));
  return 0;
}

// The small-scalar split of a ThresholdAggregate's Lagrange coefficients (ta_small.h): c[0..t)
// and s (32 B big-endian, canonical); returns 1 if the split applies.
extern "C" int hc_ta_small(const int64_t* idx, int t, int64_t* c, uint8_t* s32) {
  Fr s;
  if (!ta_small_split(idx, t, c, s)) return 0;
  fr_to_be(s32, fr_from_mont(s));
  return 1;
}

// ThresholdAggregate through the small-scalar split: [s] (sum_j [c_j] sigma_j), compressed
// (the GPU's k_ta_small / k_ta_sladder restated one lane at a time); 2 = undecodable member,
// 7 = split refused.
extern "C" int hc_lagrange_g2_small(const uint8_t* sigs, const int64_t* idx, int k, uint8_t* out96) {
  int64_t c[TA_SMALL_MAX];
  Fr s;
  if (!ta_small_split(idx, k, c, s)) return 7;
  G2J q = jac_infinity<Fp2>();
  for (int i = 0; i < k; i++) {
    G2A a;
    if (g2_decompress(a, sigs + 96 * i)) return ST_BAD_SIGNATURE;
    const uint64_t m = c[i] < 0 ? (uint64_t)(-c[i]) : (uint64_t)c[i];
    const uint32_t mw[2] = {(uint32_t)m, (uint32_t)(m >> 32)};
    G2J t = jac_mul_aff(a, mw, 64);
    if (c[i] < 0) t = jac_neg(t);
    q = jac_add(q, t);
  }
  const Fr sc = fr_from_mont(s);
  const G2A qa = jac_to_aff(q);
  g2_compress(out96, jac_to_aff(qa.inf ? jac_infinity<Fp2>() : jac_mul_aff(qa, sc.v, 256)));
  return 0;
}

// the G1 subgroup test both ways for an affine point given as big-endian x || y (on the curve,
// not checked): out[0] = ec.h g1_in_subgroup (stored words), out[1] = ec28.h lazy limbs,
// out[2] = the Fp products the lazy test spent
extern "C" int hc_g1_subgroup2(const uint8_t* xy96, int* out) {
  Fp xr, yr;
  fp_from_be_raw(xr, xy96);
  fp_from_be_raw(yr, xy96 + 48);
  const G1A p = {fp_to_mont(xr), fp_to_mont(yr), false};
  out[0] = g1_in_subgroup(p) ? 1 : 0;
  g_cnt_fp_mul = 0;
  out[1] = g1_in_subgroup28(p) ? 1 : 0;
  out[2] = (int)g_cnt_fp_mul;
  return 0;
}

// the G2 subgroup test both ways, affine point as big-endian x0 || x1 || y0 || y1 (on the twist,
// not checked): out[0] = ec.h g2_in_subgroup, out[1] = ec28.h lazy limbs, out[2] = its Fp products
extern "C" int hc_g2_subgroup2(const uint8_t* xy192, int* out) {
  Fp w[4];
  for (int i = 0; i < 4; i++) {
    Fp r;
    fp_from_be_raw(r, xy192 + 48 * i);
    w[i] = fp_to_mont(r);
  }
  const G2A q = {{w[0], w[1]}, {w[2], w[3]}, false};
  out[0] = g2_in_subgroup(q) ? 1 : 0;
  g_cnt_fp_mul = 0;
  out[1] = g2_in_subgroup28(q) ? 1 : 0;
  out[2] = (int)g_cnt_fp_mul;
  return 0;
}

// ec28.h zero tests on a 14-limb value: out[0] = l_is_zero (carries + k p comparison),
// out[1] = l_is_zero_mul (the Montgomery product by 1)
extern "C" int hc_l28_is_zero(const uint32_t* limbs, int* out) {
  L28 a;
  for (int i = 0; i < 14; i++) a.l[i] = limbs[i];
  out[0] = l_is_zero(a) ? 1 : 0;
  out[1] = l_is_zero_mul(a) ? 1 : 0;
  return 0;
}

// sum over k items of [a_i + b_i lambda] pk_i through ec28.h's lazy chunk ladder (the table built
// as vbatch.hip k_rlc_msm builds it: P, phi(P), P + phi(P) affine), compressed
extern "C" int hc_rlc_sum_g1_lazy(int k, const uint8_t* pks, const uint32_t* ab, uint8_t* out48) {
  struct Pair {
    uint32_t x, y;
  };
  G1J tab[3 * 64];
  Pair coef[64];
  if (k > 64) return 1;
  for (int i = 0; i < k; i++) {
    G1A p;
    if (g1_decompress(p, pks + 48 * i)) return 1;
    const G1A p2 = {fp_mul(p.x, fp_from_const(G1_BETA)), p.y, false};
    const G1A p3 = jac_to_aff(jac_add_aff(jac_from_aff(p), p2));
    tab[3 * i] = jac_from_aff(p);
    tab[3 * i + 1] = jac_from_aff(p2);
    tab[3 * i + 2] = jac_from_aff(p3);
    coef[i] = {ab[2 * i], ab[2 * i + 1]};
  }
  g1_compress(out48, jac_to_aff(g1l_msm_ladder(tab, coef, 0, (uint32_t)k)));
  return 0;
}

// hostmul64.h's 64-bit products against the 28-bit cores they replace on the host, on `iters`
// random operands each: stored words below 2^381, normalised limbs, lazy limbs (below 2^30; the
// dot product's below 2^29), and the Fp2 product's signed real part.  Returns the mismatches.
extern "C" int hc_mul64_selftest(int iters, uint64_t seed) {
  uint64_t s = seed * 0x9E3779B97F4A7C15ull + 1;
  auto rnd = [&]() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return (uint32_t)(s >> 16);
  };
  auto words = [&](uint32_t* w) {
    for (int i = 0; i < 12; i++) w[i] = rnd();
    w[11] &= 0x1fffffffu;  // < 2^381 < 2p
  };
  auto limbs = [&](uint32_t* l, int bits) {
    for (int i = 0; i < 14; i++) l[i] = rnd() & ((1u << bits) - 1u);
  };
  int bad = 0;
  for (int it = 0; it < iters; it++) {
    uint32_t a[12], b[12], c[12], d[12], r0[12], r1[12], q0[12], q1[12];
    words(a), words(b), words(c), words(d);
    fp_mul_core(r0, a, b);
    hm64::mul_words(q0, a, b);
    bad += memcmp(r0, q0, sizeof r0) != 0;
    fp_sqr_core(r0, a);
    hm64::mul_words(q0, a, a);
    bad += memcmp(r0, q0, sizeof r0) != 0;
    fp2_mul_core(r0, r1, a, b, c, d);
    hm64::fp2_mul_words(q0, q1, a, b, c, d);
    bad += memcmp(r0, q0, sizeof r0) != 0 || memcmp(r1, q1, sizeof r1) != 0;
    fp2_sqr_core(r0, r1, a, b);
    hm64::fp2_mul_words(q0, q1, a, b, a, b);
    bad += memcmp(r0, q0, sizeof r0) != 0 || memcmp(r1, q1, sizeof r1) != 0;
    uint32_t x[14], y[14], z[14], u[14], l0[14], l1[14], m0[14], m1[14];
    for (int lazy = 0; lazy < 2; lazy++) {
      limbs(x, lazy ? 30 : 28), limbs(y, lazy ? 30 : 28);
      fp_mul28_core(l0, x, y);
      hm64::mul_limbs28(m0, x, y);
      bad += memcmp(l0, m0, sizeof l0) != 0;
      fp_sqr28_core(l0, x);
      hm64::mul_limbs28(m0, x, x);
      bad += memcmp(l0, m0, sizeof l0) != 0;
      limbs(x, 29), limbs(y, 29), limbs(z, 29), limbs(u, 29);
      f2l_dot_core(l0, x, y, z, u);
      hm64::dot_limbs28(m0, x, y, z, u);
      bad += memcmp(l0, m0, sizeof l0) != 0;
    }
    limbs(x, 28), limbs(y, 28), limbs(z, 28), limbs(u, 28);
    F2L fa, fb;
    for (int i = 0; i < 14; i++) fa.c0.l[i] = x[i], fa.c1.l[i] = y[i], fb.c0.l[i] = z[i], fb.c1.l[i] = u[i];
    f2l_mul_core(l0, l1, x, y, z, u);
    const F2L fr = f2l_mul(fa, fb);
    for (int i = 0; i < 14; i++) m0[i] = fr.c0.l[i], m1[i] = fr.c1.l[i];
    bad += memcmp(l0, m0, sizeof l0) != 0 || memcmp(l1, m1, sizeof l1) != 0;
    // the paired leaves' core (ec28.h mul28x2_core, the G1 formulas): two products / squares at once
    for (int lazy = 0; lazy < 2; lazy++) {
      limbs(x, lazy ? 30 : 28), limbs(y, lazy ? 30 : 28), limbs(z, lazy ? 30 : 28), limbs(u, lazy ? 30 : 28);
      mul28x2_core<false>(l0, l1, x, y, z, u);
      hm64::mul_limbs28(m0, x, y);
      hm64::mul_limbs28(m1, z, u);
      bad += memcmp(l0, m0, sizeof l0) != 0 || memcmp(l1, m1, sizeof l1) != 0;
      mul28x2_core<true>(l0, l1, x, x, z, z);
      hm64::mul_limbs28(m0, x, x);
      hm64::mul_limbs28(m1, z, z);
      bad += memcmp(l0, m0, sizeof l0) != 0 || memcmp(l1, m1, sizeof l1) != 0;
    }
  }
  return bad;
}

// the sparse-format chunk ladders (ec28.h g1l/g2l_msm_ladder_sparse) with the table built as
// vbatch.hip k_rlc_msm builds it (rlc.h sparse_put / sparse_fix): sum over k items of
// [A_i + B_i lambda] P_i, dig = 4 words per item (word 3 = 0: the item is skipped), compressed
struct HcQuad {
  uint32_t x, y, z, w;
};
extern "C" int hc_rlc_sum_g1_sparse(int k, const uint8_t* pks, const uint32_t* dig, uint8_t* out48) {
  G1J tab[4 * 64];
  HcQuad coef[64];
  if (k < 1 || k > 64) return 1;
  Fp acc = fp_one();
  for (int i = 0; i < k; i++) {
    G1A p;
    if (g1_decompress(p, pks + 48 * i)) return 1;
    acc = sparse_put(tab, (uint64_t)i, p, G1A{fp_mul(p.x, fp_from_const(G1_BETA)), p.y, false}, acc);
    coef[i] = {dig[4 * i], dig[4 * i + 1], dig[4 * i + 2], dig[4 * i + 3]};
  }
  Fp inv = fp_inv(acc);
  for (int i = k - 1; i >= 0; i--) inv = sparse_fix(tab, (uint64_t)i, inv);
  g1_compress(out48, jac_to_aff(g1l_msm_ladder_sparse(tab, coef, 0, (uint32_t)k)));
  return 0;
}
extern "C" int hc_rlc_sum_g2_sparse(int k, const uint8_t* sigs, const uint32_t* dig, uint8_t* out96) {
  G2J tab[4 * 64];
  HcQuad coef[64];
  if (k < 1 || k > 64) return 1;
  Fp2 acc = f2_one();
  for (int i = 0; i < k; i++) {
    G2A p;
    if (g2_decompress(p, sigs + 96 * i)) return 1;
    const G2A p2 = {f2_mul(p.x, f2_from_const(PSI2_CX)), f2_neg(f2_mul(p.y, f2_from_const(PSI2_CY))), false};
    acc = sparse_put(tab, (uint64_t)i, p, p2, acc);
    coef[i] = {dig[4 * i], dig[4 * i + 1], dig[4 * i + 2], dig[4 * i + 3]};
  }
  Fp2 inv = f2_inv(acc);
  for (int i = k - 1; i >= 0; i--) inv = sparse_fix(tab, (uint64_t)i, inv);
  g2_compress(out96, jac_to_aff(g2l_msm_ladder_sparse(tab, coef, 0, (uint32_t)k)));
  return 0;
}

// [|x|] P both ways for a Jacobian G2 point given as the affine point (x0 x1 y0 y1, big-endian)
// scaled by z = (z0, z1) (z = 0: infinity): out96x2 = compressed results of ec.h jac_mul_by_xabs
// and ec28.h g2l_mul_by_xabs_l
extern "C" int hc_g2_mul_xabs2(const uint8_t* xyz288, uint8_t* out192) {
  Fp w[6];
  for (int i = 0; i < 6; i++) {
    Fp r;
    fp_from_be_raw(r, xyz288 + 48 * i);
    w[i] = fp_to_mont(r);
  }
  const Fp2 x = {w[0], w[1]}, y = {w[2], w[3]}, z = {w[4], w[5]};
  const Fp2 z2 = f2_sqr(z);
  const G2J P = {f2_mul(x, z2), f2_mul(y, f2_mul(z2, z)), z};
  g2_compress(out192, jac_to_aff(jac_mul_by_xabs(P)));
  g2_compress(out192 + 96, jac_to_aff(g2l_mul_by_xabs_l([&]() { return P; })));
  return 0;
}

// sum over k items of [a_i + b_i lambda] S_i (G2) through ec28.h's lazy chunk ladder, the table
// as k_rlc_msm builds it (S, -psi^2(S), S - psi^2(S) affine), compressed
extern "C" int hc_rlc_sum_g2_lazy(int k, const uint8_t* sigs, const uint32_t* ab, uint8_t* out96) {
  struct Pair {
    uint32_t x, y;
  };
  G2J tab[3 * 64];
  Pair coef[64];
  if (k > 64) return 1;
  for (int i = 0; i < k; i++) {
    G2A p;
    if (g2_decompress(p, sigs + 96 * i)) return 1;
    const G2A p2 = {f2_mul(p.x, f2_from_const(PSI2_CX)), f2_neg(f2_mul(p.y, f2_from_const(PSI2_CY))), false};
    const G2A p3 = jac_to_aff(jac_add_aff(jac_from_aff(p), p2));
    tab[3 * i] = jac_from_aff(p);
    tab[3 * i + 1] = jac_from_aff(p2);
    tab[3 * i + 2] = jac_from_aff(p3);
    coef[i] = {ab[2 * i], ab[2 * i + 1]};
  }
  g2_compress(out96, jac_to_aff(g2l_msm_ladder(tab, coef, 0, (uint32_t)k)));
  return 0;
}

// ---- round 4: the Miller-loop arithmetic in lazy limbs (pair28.h) against the stored-word code
static Fp hc_fp_in(const uint8_t* b) {
  Fp r;
  fp_from_be_raw(r, b);
  return fp_to_mont(r);
}
static void hc_fp_out(uint8_t* b, const Fp& a) { fp_to_be_raw(b, fp_from_mont(a)); }
static void hc_f2_out(uint8_t* b, const Fp2& a) {
  hc_fp_out(b, a.c0);
  hc_fp_out(b + 48, a.c1);
}

// The 68 lines of Q (x0 x1 y0 y1, canonical big-endian) by lines.h's stored-word chain and by
// pair28.h line_chain28, canonical bytes (68 x 288 each); cnt: Fp products of each chain.
extern "C" int hc_line_chain28(const uint8_t* q192, int eval, uint8_t* out_stored, uint8_t* out_lazy,
                               unsigned long long* cnt) {
  const G2A Q = {{hc_fp_in(q192), hc_fp_in(q192 + 48)}, {hc_fp_in(q192 + 96), hc_fp_in(q192 + 144)}, false};
  LineEntryHost ls[N_LINES];
  g_cnt_fp_mul = 0;
  hc_line_chain(Q, ls, eval != 0);
  cnt[0] = g_cnt_fp_mul;
  for (int j = 0; j < N_LINES; j++) {
    hc_f2_out(out_stored + 288 * j, ls[j].a0);
    hc_f2_out(out_stored + 288 * j + 96, ls[j].a1);
    hc_f2_out(out_stored + 288 * j + 192, ls[j].b1);
  }
  g_cnt_fp_mul = 0;
  LineCoeffs ll[N_LINES];
  auto put = [&](int j, const LineCoeffs& l) { ll[j] = l; };
  if (eval) line_chain28<true>([&]() { return Q; }, put);
  else line_chain28<false>([&]() { return Q; }, put);
  cnt[1] = g_cnt_fp_mul;
  int bad = 0;
  for (int j = 0; j < N_LINES; j++) {
    // reduced values join to stored words below 2p: check the stored-word invariant too
    const Fp* v[6] = {&ll[j].a0.c0, &ll[j].a0.c1, &ll[j].a1.c0, &ll[j].a1.c1, &ll[j].b1.c0, &ll[j].b1.c1};
    for (int k = 0; k < 6; k++) {
      Fp d;
      if (raw_sub_const(d, *v[k], P2_RAW) == 0) bad = 1;  // >= 2p
      hc_fp_out(out_lazy + 288 * j + 48 * k, *v[k]);
    }
  }
  return bad;
}

// The three-lane Fp12 operations of pair28.h (g4_sqr / g4_mul_line, the roles run one after the
// other with the exchanges of pair3.h's Grp) against tower.h's f12_sqr / f12_mul_line.  f: 12 Fp in
// tower order (c0.c0, c0.c1, c0.c2, c1.c0, c1.c1, c1.c2; Fp2 as c0, c1); line: a0, a1, b1.  out:
// four Fp12 values, 576 B each: lanes' square, tower square, lanes' line product, tower line product.
extern "C" int hc_g4_ops(const uint8_t* f576, const uint8_t* line288, uint8_t* out) {
  Fp12 f;
  Fp2* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
  for (int i = 0; i < 6; i++) *c[i] = {hc_fp_in(f576 + 96 * i), hc_fp_in(f576 + 96 * i + 48)};
  const Fp2 a0 = {hc_fp_in(line288), hc_fp_in(line288 + 48)}, a1 = {hc_fp_in(line288 + 96), hc_fp_in(line288 + 144)},
            b1 = {hc_fp_in(line288 + 192), hc_fp_in(line288 + 240)};
  // lane k = (z_k, z_{k+3}) with z = (c0.c0, c1.c0, c0.c1, c1.c1, c0.c2, c1.c2); pair3.h g_from_f12
  const Fp2 z[6] = {f.c0.c0, f.c1.c0, f.c0.c1, f.c1.c1, f.c0.c2, f.c1.c2};
  F4L A[3];
  for (int k = 0; k < 3; k++) A[k] = f4l_red(f4l_from(z[k], z[k + 3]));
  const int P_[3] = {1, 0, 0}, Q_[3] = {2, 1, 2}, E_[3] = {0, 2, 1};
  auto out12 = [](uint8_t* b, const F4L* L) {
    Fp2 zz[6];
    for (int k = 0; k < 3; k++) {
      zz[k] = f2l_join(L[k].x);
      zz[k + 3] = f2l_join(L[k].y);
    }
    const Fp2 t[6] = {zz[0], zz[2], zz[4], zz[1], zz[3], zz[5]};  // back to tower order
    for (int i = 0; i < 6; i++) hc_f2_out(b + 96 * i, t[i]);
  };
  auto out12t = [](uint8_t* b, const Fp12& g) {
    const Fp2 t[6] = {g.c0.c0, g.c0.c1, g.c0.c2, g.c1.c0, g.c1.c1, g.c1.c2};
    for (int i = 0; i < 6; i++) hc_f2_out(b + 96 * i, t[i]);
  };
  F4L v[3], w[3], C[3];
  for (int k = 0; k < 3; k++) g4_sqr_p1(A[k], A[P_[k]], A[Q_[k]], v[k], w[k]);
  for (int k = 0; k < 3; k++) C[k] = g4_sqr_p2(k, w[k], v[P_[k]], v[Q_[k]], v[E_[k]]);
  out12(out, C);
  out12t(out + 576, f12_sqr(f));
  const F2L la0 = f2l_from(a0), la1 = f2l_from(a1), lb1 = f2l_from(b1);
  F4L Qn[3];
  for (int k = 0; k < 3; k++) Qn[k] = g4_line_p1(A[k], la1);
  for (int k = 0; k < 3; k++) C[k] = g4_line_p2(k, A[k], la0, lb1, Qn[(k + 1) % 3]);
  out12(out + 1152, C);
  out12t(out + 1728, f12_mul_line(f, a0, a1, b1));
  return 0;
}

// pair28.h's final exponentiation in lazy limbs, the three roles emulated (F2One), against
// pairing.h final_exponentiation: f576 tower order (as hc_g4_ops); out: both results (576 + 576)
extern "C" int hc_fe28(const uint8_t* f576, uint8_t* out) {
  Fp12 f;
  Fp2* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
  for (int i = 0; i < 6; i++) *c[i] = {hc_fp_in(f576 + 96 * i), hc_fp_in(f576 + 96 * i + 48)};
  auto lanes = [](const Fp12& g, F4L* A) {
    const Fp2 z[6] = {g.c0.c0, g.c1.c0, g.c0.c1, g.c1.c1, g.c0.c2, g.c1.c2};
    for (int k = 0; k < 3; k++) A[k] = f4l_red(f4l_from(z[k], z[k + 3]));
  };
  auto tower = [](const F4L* L) {
    Fp2 z[6];
    for (int k = 0; k < 3; k++) {
      z[k] = f2l_join(L[k].x);
      z[k + 3] = f2l_join(L[k].y);
    }
    Fp12 g;
    g.c0 = {z[0], z[2], z[4]};
    g.c1 = {z[1], z[3], z[5]};
    return g;
  };
  const int P_[3] = {1, 0, 0}, Q_[3] = {2, 1, 2}, E_[3] = {0, 2, 1};
  struct L3 {
    F4L v[3];
  };
  auto cyc = [&](const L3& A) {
    L3 t, r;
    for (int k = 0; k < 3; k++) t.v[k] = g4_cyc_p1(A.v[k]);
    for (int k = 0; k < 3; k++) r.v[k] = g4_cyc_p2(k, t.v[E_[k]], A.v[k]);
    return r;
  };
  auto mul = [&](const L3& A, const L3& B) {
    L3 v, w, r;
    for (int k = 0; k < 3; k++)
      g4_mul_p1(A.v[k], B.v[k], f4l_add(A.v[P_[k]], A.v[Q_[k]]), f4l_add(B.v[P_[k]], B.v[Q_[k]]), v.v[k], w.v[k]);
    for (int k = 0; k < 3; k++) r.v[k] = g4_sqr_p2(k, w.v[k], v.v[P_[k]], v.v[Q_[k]], v.v[E_[k]]);
    return r;
  };
  auto conj = [&](const L3& A) {
    L3 r;
    for (int k = 0; k < 3; k++) r.v[k] = g4_conj(k, A.v[k]);
    return r;
  };
  auto frob1 = [&](const L3& A) {
    L3 r;
    for (int k = 0; k < 3; k++) r.v[k] = g4_frob<1>(k, A.v[k]);
    return r;
  };
  auto frob2 = [&](const L3& A) {
    L3 r;
    for (int k = 0; k < 3; k++) r.v[k] = g4_frob<2>(k, A.v[k]);
    return r;
  };
  auto pow_x = [&](const L3& F) {
    L3 r = F;
    for (int i = 62; i >= 0; i--) {
      r = cyc(r);
      if ((HB_X_ABS >> i) & 1) r = mul(r, F);
    }
    return conj(r);
  };
  L3 F, I;
  lanes(f, F.v);
  // the inversion in stored words (pair3.h g_inv's result is the group's f^-1; the tower's here)
  lanes(f12_inv(tower(F.v)), I.v);
  L3 t = mul(conj(F), I);
  t = mul(frob2(t), t);
  L3 x = t, b = t;
  for (int st = 0; st < 5; st++) {
    const L3 px = pow_x(x);
    if (st == 3) b = x;
    if (st < 2) x = mul(px, conj(x));
    else if (st == 2) x = mul(px, frob1(x));
    else x = px;
  }
  const L3 cc = mul(mul(x, frob2(b)), conj(b));
  const L3 res = mul(cc, mul(cyc(t), t));
  const Fp12 got = tower(res.v), want = final_exponentiation(f);
  const Fp2 g6[6] = {got.c0.c0, got.c0.c1, got.c0.c2, got.c1.c0, got.c1.c1, got.c1.c2};
  const Fp2 w6[6] = {want.c0.c0, want.c0.c1, want.c0.c2, want.c1.c0, want.c1.c1, want.c1.c2};
  for (int i = 0; i < 6; i++) {
    hc_f2_out(out + 96 * i, g6[i]);
    hc_f2_out(out + 576 + 96 * i, w6[i]);
  }
  return 0;
}

// fp.h fp_inv (divsteps, early exit) and fp_inv_ct (fixed trip count, the secret-key paths)
// against fp_inv_pow (a^(p-2)): x canonical big-endian; out: the three inverses (canonical), the
// batches each divstep version ran
extern "C" int hc_fp_inv(const uint8_t* x48, uint8_t* out144, int* batches, int* batches_ct) {
  const Fp a = hc_fp_in(x48);
  hc_fp_out(out144, fp_inv(a, batches));
  hc_fp_out(out144 + 48, fp_inv_pow(a));
  hc_fp_out(out144 + 96, fp_inv_ct(a, batches_ct));
  return 0;
}

// coalesce.h's state machine with a stub batch runner (no GPU): `threads` callers each submit
// `reqs` requests of 1..3 items; the runner sleeps run_us, checks that none of its requests ran
// before and writes each item's status (request id & 0xff).  out[0]: most batches running at once
// (counted by the runner), out[1]: batches, out[2]: requests run twice or never, out[3]: wrong
// statuses, out[4]: the coalescer's own max_active.
#include "../../charon_amd/csrc/coalesce.h"
extern "C" int hc_coalesce_stress(int threads, int reqs, int inflight, int window_us, int run_us, int* out) {
  Coalescer c;
  CoalesceParams p;
  p.us = (size_t)window_us;
  p.max_items = 1u << 16;
  p.inflight = (size_t)inflight;
  const int total = threads * reqs;
  std::vector<std::atomic<int>> runs(total);
  for (auto& r : runs) r = 0;
  std::atomic<int> running{0}, max_running{0}, bad_status{0};
  auto run = [&](std::vector<VReq*>& batch) {
    const int now = ++running;
    int m = max_running.load();
    while (now > m && !max_running.compare_exchange_weak(m, now)) {
    }
    std::this_thread::sleep_for(std::chrono::microseconds(run_us));
    for (VReq* r : batch) {
      const int id = (int)(intptr_t)r->pk;  // the request id travels in the pk pointer
      runs[id]++;
      for (size_t i = 0; i < r->n; i++) r->st[i] = (uint8_t)(id & 0xff);
      r->rc = 0;
    }
    --running;
  };
  std::vector<std::thread> th;
  for (int t = 0; t < threads; t++)
    th.emplace_back([&, t] {
      for (int k = 0; k < reqs; k++) {
        const int id = t * reqs + k;
        uint8_t st[3] = {0xee, 0xee, 0xee};
        VReq me;
        me.pk = (const uint8_t*)(intptr_t)id;
        me.n = 1 + (size_t)(id % 3);
        me.st = st;
        coalesce_submit(c, p, me, run);
        for (size_t i = 0; i < me.n; i++)
          if (st[i] != (uint8_t)(id & 0xff)) bad_status++;
        if (!me.done) bad_status++;
      }
    });
  for (auto& x : th) x.join();
  int wrong_runs = 0;
  for (auto& r : runs)
    if (r.load() != 1) wrong_runs++;
  out[0] = max_running.load();
  out[1] = (int)c.batches;
  out[2] = wrong_runs;
  out[3] = bad_status.load();
  out[4] = c.max_active;
  return 0;
}

// pipeline.hip k_lines_at_p's line (the lazy chain evaluated at a variable P inside the chain)
// against k_lines_msg + k_mml_eval (the unevaluated lazy chain, then a1 x_P, b1 y_P by stored-word
// products): q192 = Q (x0 x1 y0 y1), p96 = P (x y), canonical big-endian.  out: 68 x 288 B each,
// canonical; returns 1 if a line at P is not below 2p (the multi-Miller loop's input bound).
extern "C" int hc_lines_at_p(const uint8_t* q192, const uint8_t* p96, uint8_t* out_at_p, uint8_t* out_eval) {
  const G2A Q = {{hc_fp_in(q192), hc_fp_in(q192 + 48)}, {hc_fp_in(q192 + 96), hc_fp_in(q192 + 144)}, false};
  const Fp px = hc_fp_in(p96), py = hc_fp_in(p96 + 48);
  const L28 xp = l_from(px), yp = l_from(py);
  LineCoeffs la[N_LINES], lu[N_LINES];
  line_chain28_st([&]() { return Q; },
                  [&](const Line28& l) {
                    return LineCoeffs{f2l_join(l.a0), {l_join(l_mul(l.a1.c0, xp)), l_join(l_mul(l.a1.c1, xp))},
                                      {l_join(l_mul(l.b1.c0, yp)), l_join(l_mul(l.b1.c1, yp))}};
                  },
                  [&](int j, const LineCoeffs& c) { la[j] = c; });
  line_chain28<false>([&]() { return Q; }, [&](int j, const LineCoeffs& c) { lu[j] = c; });
  int bad = 0;
  for (int j = 0; j < N_LINES; j++) {
    const Fp2 e1 = f2_mul_fp(lu[j].a1, px), e2 = f2_mul_fp(lu[j].b1, py);
    hc_f2_out(out_eval + 288 * j, lu[j].a0);
    hc_f2_out(out_eval + 288 * j + 96, e1);
    hc_f2_out(out_eval + 288 * j + 192, e2);
    const Fp* v[6] = {&la[j].a0.c0, &la[j].a0.c1, &la[j].a1.c0, &la[j].a1.c1, &la[j].b1.c0, &la[j].b1.c1};
    for (int k = 0; k < 6; k++) {
      Fp d;
      if (raw_sub_const(d, *v[k], P2_RAW) == 0) bad = 1;
      hc_fp_out(out_at_p + 288 * j + 48 * k, *v[k]);
    }
  }
  return bad;
}

// msgtable.h: the distinct messages of n items by the sequential dedup (threads 0) or the parallel
// one (threads 4 / 8).  idx: each item's id; returns the number of distinct messages, or -1 if a
// table entry's bytes differ from an item it names.
#include "../../charon_amd/csrc/msgtable.h"
extern "C" long hc_dedup(const uint8_t* msgs, const uint64_t* off, const uint32_t* len, size_t n, int threads,
                         uint32_t* idx) {
  MsgTable t;
  if (threads) dedup_messages_par(msgs, off, len, n, t, (unsigned)threads);
  else dedup_messages(msgs, off, len, n, nullptr, t);
  for (size_t k = 0; k < n; k++) {
    const uint32_t id = t.idx[k];
    idx[k] = id;
    if (id >= t.len.size() || t.len[id] != len[k] || memcmp(t.bytes.data() + t.off[id], msgs + off[k], len[k]) != 0)
      return -1;
  }
  return (long)t.len.size();
}
