// TEST-ONLY harness: compiles the kernels' per-item arithmetic (charon_amd/csrc/*.h) for the
// host CPU so tests/test_hostcheck.py can compare it with the Python oracle without a GPU.
// The product library (libhipbls.so) never loads this; it is not a fallback.
// Built with HB_COUNT_OPS: every Fp / Fr Montgomery product bumps a thread-local counter, which
// hc_count_* read to freeze the algorithmic work per item (charon_amd/opcounts.py).
#define HB_COUNT_OPS 1
#include "../../charon_amd/csrc/ops.h"
#include <string.h>

namespace hb {
thread_local unsigned long long g_cnt_fp_mul = 0, g_cnt_fr_mul = 0;
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
extern "C" int hc_cpu_slot(int threads, int units, int n, int t, const uint8_t* pks, const uint8_t* sigs,
                           const uint8_t* msgs, const uint32_t* midx, const uint8_t* ta_sigs,
                           const uint8_t* root_sigs) {
  std::atomic<int> next{0}, bad{0};
  std::vector<int64_t> idx(t);
  for (int i = 0; i < t; i++) idx[i] = i + 1;
  auto work = [&]() {
    for (;;) {
      int v = next.fetch_add(1);
      if (v >= units) return;
      bool ok = true;
      for (int i = v * n; i < v * n + n; i++)
        ok &= hc_verify(pks + 48ull * i, msgs + 32ull * midx[i], 32, sigs + 96ull * i) == 0;
      uint8_t out[96];
      ok &= hc_lagrange_g2(ta_sigs + 96ull * t * v, idx.data(), t, out) == 0;
      ok &= memcmp(out, root_sigs + 96ull * v, 96) == 0;
      if (!ok) bad.fetch_add(1);
    }
  };
  std::vector<std::thread> ws;
  for (int k = 0; k < threads; k++) ws.emplace_back(work);
  for (auto& w : ws) w.join();
  return bad.load();
}
