// pipeline.hip: the staged verify kernels of libhipbls.so (tbls.Verify, herumi.go:288-304).
//
// Compiled with HB_FAST_FPMUL: every Fp product is the register-convention subroutine hb_fpmul
// (fp.h, fpmul_asm.inc) and every other field / curve / tower function is inlined, so these
// kernels make no ABI calls and keep their state in registers.  The one-lane kernels of
// hipbls.hip use the standard-convention product instead (their code is too large to inline).
#define HB_FAST_FPMUL 1
#include "layout.h"
#include "pair3.h"

namespace hb {

#if defined(__HIP_DEVICE_COMPILE__)
HB_DEFINE_FPMUL_SUBROUTINE(hb_fpmul_holder_pipeline)
#else
__global__ void hb_fpmul_holder_pipeline() {}
#endif

#define KERNEL_BOUNDS __launch_bounds__(64)
constexpr int BLOCK = 64;

#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ G2J xch_pair(const G2J& p) {  // the point of lane ^ 1
  G2J r;
  const uint32_t* s = reinterpret_cast<const uint32_t*>(&p);
  uint32_t* d = reinterpret_cast<uint32_t*>(&r);
  const int addr = (int)((threadIdx.x ^ 1u) << 2);
  HB_UNROLL for (int k = 0; k < (int)(sizeof(G2J) / 4); k++)
    d[k] = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)s[k]);
  return r;
}
#endif

// Two lanes per distinct message: hash_to_curve G2 (RFC 9380, DST ..._POP_), affine.  Both lanes
// expand the message; the even lane maps u0, the odd lane u1 (SSWU + 3-isogeny, the larger half
// of the work, in parallel), then the even lane adds the pair and clears the cofactor.
__global__ KERNEL_BOUNDS void k_hash_to_g2(const uint8_t* __restrict__ msgs, const uint64_t* __restrict__ off,
                                           const uint32_t* __restrict__ len, uint32_t n, MsgEntry* __restrict__ hm) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t i = t >> 1;
  const bool odd = (t & 1u) != 0;
  const uint32_t ii = i < n ? i : n - 1;  // every lane takes part in the exchange
  Fp2 u0, u1;
  hash_to_field_fp2(u0, u1, msgs + off[ii], len[ii]);
  Fp2 x, y;
  sswu_map(x, y, odd ? u1 : u0);
  const G2J q = iso3_map(x, y);
  const G2J q1 = xch_pair(q);
  if (odd || i >= n) return;
  G2A h = jac_to_aff(g2_clear_cofactor(jac_add(q, q1)));
  HmEntry e;
  e.x = h.x;
  e.y = h.y;
  e.inf = h.inf ? 1u : 0u;
  e.pad[0] = e.pad[1] = e.pad[2] = 0;
  hm[i].h = e;
#endif
}

// The Miller chain of an affine G2 point Q: 68 lines, stored at out[j * stride].  EVAL: evaluate
// each line at -g1 (pair (-g1, sig) of the verification equation); otherwise store (a0, c1, c2).
template <bool EVAL>
__device__ __forceinline__ void line_chain(const G2A& Q, LineEntry* __restrict__ out, size_t stride) {
  G2Proj T = {Q.x, Q.y, f2_one()};
  int j = 0;
  HB_NOUNROLL for (int i = 62; i >= 0; i--) {
    LineCoeffs l = miller_dbl_c(T);
    if (EVAL) line_eval(l, fp_from_const(G1_GEN_X), fp_from_const(G1_GEN_NEG_Y));
    out[(size_t)j * stride] = {l.a0, l.a1, l.b1};
    j++;
    if ((HB_X_ABS >> i) & 1) {
      l = miller_add_c(T, Q.x, Q.y);
      if (EVAL) line_eval(l, fp_from_const(G1_GEN_X), fp_from_const(G1_GEN_NEG_Y));
      out[(size_t)j * stride] = {l.a0, l.a1, l.b1};
      j++;
    }
  }
}

// One lane per distinct message: the unevaluated line chain of H(m).
__global__ KERNEL_BOUNDS void k_lines_msg(MsgEntry* __restrict__ hm, uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  line_chain<false>(hm_load(hm[i].h), hm[i].lines, 1);
}

// Verify stage 1a: one lane per partial, decompress + subgroup-check the public key
// (herumi.go:290 PublicKey.Deserialize).  A rejected key is replaced by g1 so later stages run
// the same arithmetic on well-formed values; its status byte decides the verdict.
__global__ KERNEL_BOUNDS void k_dec_pk(const uint8_t* __restrict__ pks, uint32_t n, G1AEntry* __restrict__ out,
                                       uint8_t* __restrict__ st) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G1A p;
  uint8_t bad = g1_decompress(p, pks + 48ull * i);
  if (bad) p = g1_generator();
  G1AEntry e;
  e.x = p.x;
  e.y = p.y;
  e.inf = p.inf ? 1u : 0u;
  e.pad[0] = e.pad[1] = e.pad[2] = 0;
  out[i] = e;
  st[i] = bad;
}

// Verify stage 1b: one lane per partial, decompress + subgroup-check the signature
// (herumi.go:295 Sign.Deserialize), then its Miller chain evaluated at -g1.
__global__ KERNEL_BOUNDS void k_dec_sig_lines(const uint8_t* __restrict__ sigs, uint32_t n, uint8_t* __restrict__ inf,
                                              uint8_t* __restrict__ st, LineEntry* __restrict__ lines) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G2A q;
  uint8_t bad = g2_decompress(q, sigs + 96ull * i);
  st[i] = bad;
  inf[i] = (!bad && q.inf) ? 1 : 0;
  // rejected / infinity signatures: the chain runs on whatever was decoded (integer arithmetic
  // cannot fault) and the status bytes decide the verdict
  line_chain<true>(q, lines + i, n);
}

// Verify stage 2: THREE lanes per partial (pair3.h): Miller loop over the streamed lines of
// (pk, H(m)) and (-g1, sig), final exponentiation, verdict (herumi.go:299 VerifyByte).
__global__ __launch_bounds__(64, 2) void k_pair3(const G1AEntry* __restrict__ pk, const uint8_t* __restrict__ pk_st,
                                      const uint8_t* __restrict__ sig_inf, const uint8_t* __restrict__ sig_st,
                                      const uint32_t* __restrict__ msg_idx, const MsgEntry* __restrict__ hm,
                                      const LineEntry* __restrict__ sig_lines, uint32_t n, uint8_t* __restrict__ status) {
#if defined(__HIP_DEVICE_COMPILE__)
  Grp g = grp_make();
  const int grp = (int)(threadIdx.x & 63u) / 3;
  const uint32_t item = blockIdx.x * GROUPS_PER_WAVE + (uint32_t)grp;
  const bool valid = grp < GROUPS_PER_WAVE && item < n;
  const uint32_t it = valid ? item : n - 1;  // idle lanes shadow a real item (no divergence)
  const G1AEntry P = pk[it];
  const uint32_t m = msg_idx[it];
  const LineEntry* ml = hm[m].lines;
  const LineEntry* sl = sig_lines + it;
  // Lines in loop order: for each bit i = 62..0 of |x| a doubling line (preceded by f^2 except
  // at the top) and, if bit i is set, an addition line.  One copy of the line products.
  Fp4 f = g_one(g);
  int bit = 62;
  bool pending_add = false;
  HB_NOUNROLL for (int j = 0; j < N_LINES; j++) {
    const bool dbl = !pending_add;
    if (dbl && j > 0) f = g_sqr(g, f);
    LineEntry L = ml[j];
    f = g_mul_line(g, f, L.a0, f2_mul_fp(L.a1, P.x), f2_mul_fp(L.b1, P.y));
    LineEntry S = sl[(size_t)j * n];
    f = g_mul_line(g, f, S.a0, S.a1, S.b1);
    if (dbl) {
      pending_add = ((HB_X_ABS >> bit) & 1) != 0;
      bit--;
    } else {
      pending_add = false;
    }
  }
  f = g_final_exp(g, f);
  const bool one = g_is_one(g, f);
  if (valid && g.k == 0) {
    uint8_t s;
    if (pk_st[item]) s = ST_BAD_PUBKEY;
    else if (sig_st[item]) s = ST_BAD_SIGNATURE;
    else if (P.inf || sig_inf[item] || hm[m].h.inf) s = ST_NOT_VERIFIED;  // verify_core (ops.h)
    else s = one ? ST_OK : ST_NOT_VERIFIED;
    status[item] = s;
  }
#endif
}


static inline unsigned blocks_for(size_t n) { return (unsigned)((n + BLOCK - 1) / BLOCK); }

void launch_hash_to_g2(const uint8_t* msgs, const uint64_t* off, const uint32_t* len, uint32_t n, MsgEntry* hm,
                       hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_hash_to_g2, dim3(blocks_for(2 * (size_t)n)), dim3(BLOCK), 0, s, msgs, off, len, n, hm);
}
void launch_lines_msg(MsgEntry* hm, uint32_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_lines_msg, dim3(blocks_for(n)), dim3(BLOCK), 0, s, hm, n);
}
void launch_dec_pk(const uint8_t* pks, uint32_t n, G1AEntry* out, uint8_t* st, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_dec_pk, dim3(blocks_for(n)), dim3(BLOCK), 0, s, pks, n, out, st);
}
void launch_dec_sig_lines(const uint8_t* sigs, uint32_t n, uint8_t* inf, uint8_t* st, LineEntry* lines,
                          hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_dec_sig_lines, dim3(blocks_for(n)), dim3(BLOCK), 0, s, sigs, n, inf, st, lines);
}
void launch_pair3(const G1AEntry* pk, const uint8_t* pk_st, const uint8_t* sig_inf, const uint8_t* sig_st,
                  const uint32_t* msg_idx, const MsgEntry* hm, const LineEntry* sig_lines, uint32_t n,
                  uint8_t* status, hipStream_t s) {
  if (!n) return;
  unsigned grid = (unsigned)((n + GROUPS_PER_WAVE - 1) / GROUPS_PER_WAVE);
  hipLaunchKernelGGL(k_pair3, dim3(grid), dim3(64), 0, s, pk, pk_st, sig_inf, sig_st, msg_idx, hm, sig_lines, n,
                     status);
}

}  // namespace hb
