// pipeline.hip: the Miller lines of the hashed messages and the pairing kernel of libhipbls.so
// (tbls.Verify, herumi.go:288-304).  Message hashing is in hash.hip.
//
// Compiled with HB_FAST_FPMUL: every field / curve / tower function is inlined; the Fp product and
// square are the only calls (fp.h fp_mul_leaf / fp_sqr_leaf, compiler-visible C++).
#define HB_FAST_FPMUL 1
#define HB_ARG_LANES 128  // k_lml: two-wave workgroups
#include "lines.h"
#include "pair3.h"
#include "pair6.h"

#include <stdlib.h>

namespace hb {

constexpr int BLOCK = 64;


// One lane per distinct message: the unevaluated line chain of H(m).  guard (nullable): only if
// *guard != 0 (the lines of a call that deferred them, needed only behind a failed slot-wide check)
__global__ KB_OCC(HB_OCC_LINES) void k_lines_msg(MsgEntry* __restrict__ hm, uint32_t n, const uint8_t* __restrict__ guard) {
  if (guard && *guard == 0) return;
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  line_chain_ld<false>(&hm[i].h, hm[i].lines, 1);
}

// One lane per verification group of a call whose messages have one group each (distinct
// per-validator messages, BASELINE configs[2]): the Miller chain of H(m_g) evaluated at the group's
// P_g straight into the multi-Miller loops' layout ev[j * n + g] (k_mml_eval's output) -- no
// unevaluated lines written and read back (k_lines_msg + k_mml_eval moved 68 x 288 B per message
// through HBM three times), and lanes write consecutive entries.  A unit line (1, 0, 0) for groups
// that are not READY (pk_st nonzero).  The lines are those of k_lines_msg (the same chain) times
// (1, x_P, y_P), as k_mml_eval computes them.
__global__ KB_OCC(HB_OCC_LINES) void k_lines_at_p(const G1AEntry* __restrict__ pk, const uint8_t* __restrict__ pk_st,
                                                  const uint32_t* __restrict__ msg_idx, const MsgEntry* __restrict__ hm,
                                                  uint32_t n, LineEntry* __restrict__ ev) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  LineEntry* out = ev + g;
  if (pk_st && pk_st[g]) {
    const LineEntry unit = {f2_one(), f2_zero(), f2_zero()};
    for (int j = 0; j < N_LINES; j++) out[(size_t)j * n] = unit;
    return;
  }
  const G1AEntry P = pk[g];
  const L28 xp = l_from(P.x), yp = l_from(P.y);
  const HmEntry* src = &hm[msg_idx[g]].h;
  line_chain28_st([src]() { return hm_load(*src); },
                  [&](const Line28& l) {
                    return LineCoeffs{f2l_join(l.a0), {l_join(l_mul(l.a1.c0, xp)), l_join(l_mul(l.a1.c1, xp))},
                                      {l_join(l_mul(l.b1.c0, yp)), l_join(l_mul(l.b1.c1, yp))}};
                  },
                  [&](int j, const LineCoeffs& c) { out[(size_t)j * n] = {c.a0, c.a1, c.b1}; });
#endif
}

// THREE lanes per pairing (pair3.h): Miller loop over the streamed lines of (P, H(m)) and
// (-g1, S), final exponentiation, verdict (herumi.go:299 VerifyByte).  Units and statuses as
// described at Pair3Args (layout.h).  MODE: P3_FULL as just said; P3_ML the (P, H(m)) loop only,
// stored unexponentiated; P3_FIN the (-g1, S) loop times stored values, exponentiated (the batched
// final exponentiation of vgroup.hip).
// P3_PROD: no lines, no exponentiation -- the product of a range of stored values (the
// slot-wide check's product tree).
// P3_MML: one Miller loop over the (P, H(m)) pairs of f_range consecutive entries [e f_range, ...)
// -- the squarings shared by the chunk, one sparse line product per pair and line -- stored
// unexponentiated (entries with a nonzero pk_st byte contribute one).
// P3_MLS: the (-g1, S) loop alone, stored (the final exponentiation's second factor, computed beside
// the product tree instead of in front of the exponentiation).
enum { P3_FULL = 0, P3_ML = 1, P3_FIN = 2, P3_PROD = 3, P3_MML = 4, P3_MLS = 5 };

__device__ __forceinline__ size_t f_out_index(const Pair3Args& a, uint32_t e) {
  return (size_t)e * (a.f_out_stride ? a.f_out_stride : 1u) + a.f_out_off;
}

__device__ __forceinline__ F4L f4l_load(const Fp4Entry& e) { return f4l_from(e.x, e.y); }

template <int MODE>
__global__ KB_OCC(HB_OCC_PAIR3) void k_pair3(Pair3Args a) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (a.guard && *a.guard == 0) return;
  Grp g = grp_make();
  const int grp = (int)(threadIdx.x & 63u) / 3;
  const uint32_t unit = blockIdx.x * GROUPS_PER_WAVE + (uint32_t)grp;
  uint32_t avail = a.n;
  if (a.list) {
    const uint32_t c = *a.count;
    avail = c > a.base ? c - a.base : 0;
    if (avail > a.n) avail = a.n;
  }
  if (blockIdx.x * GROUPS_PER_WAVE >= avail) return;  // wave-uniform
  const bool valid = grp < GROUPS_PER_WAVE && unit < avail;
  const uint32_t u = valid ? unit : avail - 1;  // idle lanes shadow a real unit (no divergence)
  uint32_t e = a.list ? a.list[a.base + u] : u;
  const bool agg = MODE == P3_FULL && e >= a.n_items;
  G1AEntry P{};
  uint32_t m = 0;
  const LineEntry* ml = nullptr;
  if (MODE == P3_PROD) {  // wave-uniform trip count; idle lanes multiply by one
    // (stored words: a chain of products alone, where pair28.h's per-step reductions cost more than
    // its lazy additions save -- 1.02 vs 1.13 ms per C3 slot, profiles/r04d_ab_summary.txt)
    const uint32_t first = e * a.f_range;
    const uint32_t cnt = first < a.f_n ? min(a.f_range, a.f_n - first) : 0u;
    Fp4 f = g_one(g);
    HB_NOUNROLL for (uint32_t j = 0; j < a.f_range; j++) {
      const uint32_t idx = j < cnt ? first + j : 0u;
      const Fp4Entry& v = a.f_in[3ull * idx + g.k];
      Fp4 t;
      f4_select(t, j >= cnt, Fp4{v.x, v.y}, g_one(g));
      f = g_mul(g, f, t);
    }
    if (valid) a.f_out[3 * f_out_index(a, e) + g.k] = Fp4Entry{f.x, f.y};
    return;
  }
  if (MODE == P3_MML) {  // wave-uniform trip counts; pairs past the end multiply by one
    // the lines come evaluated at each pair's P (k_mml_eval: sig_lines[j * f_n + pair], a unit line
    // for pairs that are not READY), so the three lanes of a group do not each repeat the
    // evaluation; the next (line, pair)'s load is issued before the current product (one wave per
    // SIMD: nothing else would hide its latency)
    const uint32_t first = e * a.f_range;
    const uint32_t cnt = first < a.f_n ? min(a.f_range, a.f_n - first) : 0u;
    const LineEntry* ev = a.sig_lines;
    const size_t fn = a.f_n;
    // the accumulator in lazy limbs (pair28.h g4_sqr / g4_mul_line), reduced below 2p after every
    // step; the stored-word lines are split as they are read
    F4L f = g4_one(g);
    int bit = 62;
    bool pending_add = false;
    LineEntry Ln = ev[first];
    HB_NOUNROLL for (int j = 0; j < N_LINES; j++) {
      const bool dbl = !pending_add;
      if (dbl && j > 0) f = g4_sqr(g, f);
      HB_NOUNROLL for (uint32_t k = 0; k < a.f_range; k++) {
        const LineEntry L = Ln;
        // prefetch: the next pair of this line, else the first pair of the next line
        const uint32_t k1 = k + 1 < a.f_range ? k + 1 : 0u;
        const int j1 = k + 1 < a.f_range ? j : (j + 1 < N_LINES ? j + 1 : j);
        Ln = ev[(size_t)j1 * fn + (k1 < cnt ? first + k1 : first)];
        F2L l0, l1, l2;
        line_split(L, l0, l1, l2);
        const F4L t = g4_mul_line(g, f, l0, l1, l2);
        f = f4l_select(k < cnt, f, t);
      }
      if (dbl) {
        pending_add = ((HB_X_ABS >> bit) & 1) != 0;
        bit--;
      } else {
        pending_add = false;
      }
    }
    if (valid) a.f_out[3 * f_out_index(a, e) + g.k] = f4l_store(f);
    return;
  }
  if (MODE != P3_FIN && MODE != P3_MLS) {
    P = agg ? a.agg_pk[e - a.n_items] : a.pk[e];
    m = agg ? a.agg_msg[e - a.n_items] : a.msg_idx[e];
    ml = a.hm[m].lines;
  }
  const LineEntry* sl = a.sig_lines + u;
  // Lines in loop order: for each bit i = 62..0 of |x| a doubling line (preceded by f^2 except
  // at the top) and, if bit i is set, an addition line.  One copy of the line products.  FIN without
  // sig_lines: no loop (its factors come stored, the signature side's from MLS).  The accumulator
  // and the final exponentiation in lazy limbs (pair28.h), reduced below 2p after every step.
  F4L f = g4_one(g);
  const L28 px = l_from(P.x), py = l_from(P.y);
  int bit = 62;
  bool pending_add = false;
  const int n_lines = (MODE == P3_FIN && !a.sig_lines) ? 0 : N_LINES;
  HB_NOUNROLL for (int j = 0; j < n_lines; j++) {
    const bool dbl = !pending_add;
    if (dbl && j > 0) f = g4_sqr(g, f);
    if (MODE != P3_FIN && MODE != P3_MLS) {
      F2L l0, l1, l2;
      line_split(ml[j], l0, l1, l2);
      // evaluated at P: c1 xP, c2 yP (products of reduced values: below 2p)
      f = g4_mul_line(g, f, l0, F2L{l_mul(l1.c0, px), l_mul(l1.c1, px)}, F2L{l_mul(l2.c0, py), l_mul(l2.c1, py)});
    }
    if (MODE != P3_ML) {
      F2L s0, s1, s2;
      line_split(sl[(size_t)j * a.stride], s0, s1, s2);
      f = g4_mul_line(g, f, s0, s1, s2);
    }
    if (dbl) {
      pending_add = ((HB_X_ABS >> bit) & 1) != 0;
      bit--;
    } else {
      pending_add = false;
    }
  }
  if (MODE == P3_ML) {
    const F4L r = f4l_select(a.pk_st && a.pk_st[e], f, g4_one(g));
    if (valid) a.f_out[3 * f_out_index(a, e) + g.k] = f4l_store(r);
    // groups of the small calls: the byte P3_FULL's verdict rules would fail without a pairing
    if (a.f_bad && valid && g.k == 0) a.f_bad[e] = ((a.pk_st && a.pk_st[e]) || P.inf || a.hm[m].h.inf) ? 1 : 0;
    return;
  }
  if (MODE == P3_MLS) {
    if (valid) a.f_out[3 * f_out_index(a, e) + g.k] = f4l_store(f);
    return;
  }
  if (MODE == P3_FIN) {  // times the stored Miller loops of entries [e f_range, ...) (wave-uniform trip count)
    const uint32_t first = e * a.f_range;
    const uint32_t cnt = first < a.f_n ? min(a.f_range, a.f_n - first) : 0u;
    HB_NOUNROLL for (uint32_t j = 0; j < a.f_range; j++) {
      const uint32_t idx = j < cnt ? first + j : 0u;
      f = g4_mul(g, f, f4l_select(j >= cnt, f4l_load(a.f_in[3ull * idx + g.k]), g4_one(g)));
    }
  }
  f = g4_final_exp(g, f);
  const bool one = g4_is_one(g, f);
  if (valid && g.k == 0) {
    uint8_t s;
    if (MODE == P3_FIN) s = (a.pk_st && a.pk_st[e]) ? (uint8_t)1 : (one ? ST_OK : ST_NOT_VERIFIED);
    else if (!agg && a.pk_st && a.pk_st[e]) s = ST_BAD_PUBKEY;
    else if (!agg && a.sig_st && a.sig_st[e]) s = ST_BAD_SIGNATURE;
    else if (P.inf || (!agg && a.sig_inf && a.sig_inf[e]) || a.hm[m].h.inf) s = ST_NOT_VERIFIED;  // verify_core
    else s = one ? ST_OK : ST_NOT_VERIFIED;
    if (agg) a.agg_status[e - a.n_items] = s;
    else a.status[e] = s;
  }
#endif
}

// A final exponentiation over SIX lanes per unit (pair6.h Grp6: every Fp2 product split between two
// lanes) or EIGHTEEN (pair28.h Grp18: a role's independent Fp2 products side by side over six
// lanes): the product of the unit's f_range stored values, exponentiated, its verdict -- k_pair3<FIN>
// with sig_lines == nullptr at a half / a quarter of the latency.  Ten / three units per wavefront.
#if defined(__HIP_DEVICE_COMPILE__)
template <int PER_WAVE>
__device__ __forceinline__ auto fe_group() {
  if constexpr (PER_WAVE == 3) return grp18_make();
  else return grp6_make();
}
#endif
template <int PER_WAVE>
__global__ KB_OCC(HB_OCC_PAIR3) void k_pair6_fin(Pair3Args a) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (a.guard && *a.guard == 0) return;
  const auto g = fe_group<PER_WAVE>();
  constexpr int LANES = PER_WAVE == 3 ? 18 : 6;  // lanes per unit
  const int grp = (int)(threadIdx.x & 63u) / LANES;
  if (blockIdx.x * PER_WAVE >= a.n) return;  // wave-uniform
  const uint32_t unit = blockIdx.x * PER_WAVE + (uint32_t)grp;
  const bool valid = grp < PER_WAVE && unit < a.n;
  const uint32_t e = valid ? unit : a.n - 1;
  const uint32_t first = e * a.f_range;
  const uint32_t cnt = first < a.f_n ? min(a.f_range, a.f_n - first) : 0u;
  F4L f = g4_one(g);
  HB_NOUNROLL for (uint32_t j = 0; j < a.f_range; j++) {
    const uint32_t idx = j < cnt ? first + j : 0u;
    const F4L t = f4l_select(j >= cnt, f4l_load(a.f_in[3ull * idx + g.k]), g4_one(g));
    f = j == 0 ? t : g4_mul(g, f, t);
  }
  f = g4_final_exp(g, f);  // pair28.h
  const bool one = g4_is_one(g, f);
  int sub;  // the lane of a role that stores
  if constexpr (PER_WAVE == 3) sub = g.j;
  else sub = g.h;
  if (valid && g.k == 0 && sub == 0)
    a.status[e] = (a.pk_st && a.pk_st[e]) ? (uint8_t)1 : (one ? ST_OK : ST_NOT_VERIFIED);
#endif
}

// units up to which the eighteen-lane kernel runs (HBLS_FE18_MAX at init, hbls_tune; default 256:
// a few waves per XCD; beyond, the six-lane one's fewer duplicated additions per unit win)
std::atomic<size_t> g_fe18_max{256};
static size_t fe18_max() { return g_fe18_max.load(std::memory_order_relaxed); }

void launch_pair6_fin(const Pair3Args& a, hipStream_t s) {
  if (!a.n) return;
  if (a.n <= fe18_max())
    hipLaunchKernelGGL(k_pair6_fin<3>, dim3((a.n + 2) / 3), dim3(64), 0, s, a);
  else
    hipLaunchKernelGGL(k_pair6_fin<10>, dim3((a.n + 9) / 10), dim3(64), 0, s, a);
}

// The Miller lines of every verification group's (P_g, H(m_g)) evaluated at P_g, for the
// multi-Miller loops: one lane per (line j, group g), ev[j * n + g] = (a0, a1 x_P, b1 y_P) -- a unit
// line (1, 0, 0) for groups that are not READY (pk_st nonzero), which the loop then multiplies in
// as one.  Four Fp products per line and group, once, where the three lanes of a k_pair3<MML> group
// each repeated them.
__global__ __launch_bounds__(64) void k_mml_eval(const G1AEntry* __restrict__ pk, const uint8_t* __restrict__ pk_st,
                                                 const uint32_t* __restrict__ msg_idx, const MsgEntry* __restrict__ hm,
                                                 uint32_t n, LineEntry* __restrict__ ev) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= (size_t)N_LINES * n) return;
  const uint32_t j = (uint32_t)(tid / n), g = (uint32_t)(tid % n);
  LineEntry o;
  if (pk_st && pk_st[g]) {
    o.a0 = f2_one();
    o.a1 = f2_zero();
    o.b1 = f2_zero();
  } else {
    const G1AEntry P = pk[g];
    const LineEntry L = hm[msg_idx[g]].lines[j];
    o.a0 = L.a0;
    o.a1 = f2_mul_fp(L.a1, P.x);
    o.b1 = f2_mul_fp(L.b1, P.y);
  }
  ev[tid] = o;
}

static inline unsigned blocks_for(size_t n) { return (unsigned)((n + BLOCK - 1) / BLOCK); }

void launch_mml_eval(const Pair3Args& a, LineEntry* ev, hipStream_t s) {
  const size_t n = (size_t)N_LINES * a.f_n;
  if (n) hipLaunchKernelGGL(k_mml_eval, dim3(blocks_for(n)), dim3(BLOCK), 0, s, a.pk, a.pk_st, a.msg_idx, a.hm, a.f_n, ev);
}

// The (-g1, S) Miller loop of ONE point S (Jacobian), its lines produced and consumed at once: a
// two-wave workgroup per point -- wave 0 steps T through the chain of S (affine first) and hands
// each line, evaluated at -g1, over through LDS; wave 1 squares and multiplies it into f while wave
// 0 already computes the next.  The chain's latency is then about one of the two halves instead of
// k_slines followed by k_pair3<MLS> (the slot-wide check's signature side: a tail of every slot, on
// the critical path of small slots).  bad[e] = 1 for S at infinity.
// Both halves in lazy limbs (pair28.h): the producer's chain with every Fp2 product split over a
// lane pair (ec28.h F2Half), the consumer's Fp12 over eighteen lanes (pair28.h Grp18: a role's
// independent Fp2 products side by side over six lanes) -- this kernel is latency-bound (one
// workgroup per point, few points).
// SIDE 1 (the small calls' group checks): the (P_g, H(m_g)) loop instead, H(m_g) affine from the
// message table (its lines need not exist yet: only the hashing is waited for), the lines
// evaluated at P_g by the consumer; bad[e] = the group fails without a pairing (state, P or H(m)
// at infinity), as k_pair3<ML>'s f_bad.
// (c1 x, c2 y) for a line's c1, c2 and a point's x, y (reduced), the four Fp products split over the
// pair: lane h computes the coefficient-h halves
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ void line_eval_h(F2Half m, F2L& c1, F2L& c2, const L28& x, const L28& y) {
  const bool h = m.h != 0;
  const L28 e1 = l_mul(l_pick(h, c1.c0, c1.c1), x), e2 = l_mul(l_pick(h, c2.c0, c2.c1), y);
  c1 = f2h_join(m, e1);
  c2 = f2h_join(m, e2);
}
#endif

template <int SIDE>
__global__ __launch_bounds__(128, 1) void k_lml(LmlArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (a.guard && *a.guard == 0) return;
  const uint32_t e = blockIdx.x;
  if (e >= a.n) return;  // workgroup-uniform
  __shared__ LineEntry buf[2];
  __shared__ uint32_t sinf;
  __shared__ HmEntry qsh;  // the producer's affine point, re-read at the chain's additions
  const bool producer = threadIdx.x < 64;
  const F2Half hm2 = f2half_make();
  G2P28 T;
  if (producer) {
    G2A Q;
    if (SIDE == 0) {
      const G2JEntry pe = a.pts[e];
      Q = jac_to_aff(G2J{pe.X, pe.Y, pe.Z});
    } else {
      Q = hm_load(a.hm[a.msg_idx[e]].h);
    }
    T = {f2l_from(Q.x), f2l_from(Q.y), f2l_one()};
    if (threadIdx.x == 0) {
      qsh = HmEntry{Q.x, Q.y, 0u, {0u, 0u, 0u}};
      sinf = Q.inf ? 1u : 0u;
    }
  }
  G1AEntry P{};
  if (SIDE == 1 && !producer) P = a.pk[e];
  const Grp18 g = grp18_make();
  F4L f = g4_one(g);
  const L28 px = l_from(P.x), py = l_from(P.y);  // SIDE 1: the consumer evaluates at P
  int bit = 62;  // consumer: the loop schedule of k_pair3
  bool pending_add = false;
  int pbit = 62;  // producer: the chain schedule of line_chain
  bool padd = false;
  HB_NOUNROLL for (int j = 0; j <= N_LINES; j++) {
    if (producer && j < N_LINES) {
      auto put = [&](const Line28& l28) {
        F2L c1 = l28.a1, c2 = l28.b1;
        if (SIDE == 0)  // at -g1
          line_eval_h(hm2, c1, c2, l_from(fp_from_const(G1_GEN_X)), l_from(fp_from_const(G1_GEN_NEG_Y)));
        if (threadIdx.x == 0) buf[j & 1] = {f2l_join(l28.a0), f2l_join(c1), f2l_join(c2)};
      };
      if (!padd) {
        l2_dbl_line(T, put, hm2);
        padd = ((HB_X_ABS >> pbit) & 1) != 0;
        pbit--;
      } else {
        const HmEntry qe = qsh;
        l2_add_line(T, f2l_from(qe.x), f2l_from(qe.y), put, hm2);
        padd = false;
      }
    }
    if (!producer && j > 0) {
      const LineEntry L = buf[(j - 1) & 1];
      const bool dbl = !pending_add;
      if (dbl && j > 1) f = g4_sqr(g, f);
      F2L l0, l1, l2;
      line_split(L, l0, l1, l2);
      if (SIDE == 1) line_eval_h(hm2, l1, l2, px, py);  // c1 xP, c2 yP (products of reduced values: below 2p)
      f = g4_mul_line(g, f, l0, l1, l2);
      if (dbl) {
        pending_add = ((HB_X_ABS >> bit) & 1) != 0;
        bit--;
      } else {
        pending_add = false;
      }
    }
    __syncthreads();
  }
  if (!producer && threadIdx.x < 64 + 18 && g.j == 0) {
    const size_t o = (size_t)e * (a.f_stride ? a.f_stride : 1u) + a.f_off;
    a.f_out[3 * o + g.k] = f4l_store(f);
    if (threadIdx.x == 64 && a.bad)
      a.bad[e] = SIDE == 0 ? (uint8_t)sinf : (uint8_t)((a.pk_st && a.pk_st[e]) || P.inf || sinf ? 1 : 0);
  }
#endif
}

void launch_lml(const G2JEntry* pts, uint32_t n, Fp4Entry* f_out, uint32_t f_stride, uint32_t f_off, uint8_t* bad,
                hipStream_t s, const uint8_t* guard) {
  LmlArgs a{};
  a.pts = pts;
  a.n = n;
  a.f_out = f_out;
  a.f_stride = f_stride;
  a.f_off = f_off;
  a.bad = bad;
  a.guard = guard;
  if (n) hipLaunchKernelGGL(k_lml<0>, dim3(n), dim3(128), 0, s, a);
}
void launch_lml_p(const LmlArgs& a, hipStream_t s) {
  if (a.n) hipLaunchKernelGGL(k_lml<1>, dim3(a.n), dim3(128), 0, s, a);
}

void launch_lines_msg(MsgEntry* hm, uint32_t n, hipStream_t s, const uint8_t* guard) {
  if (n) hipLaunchKernelGGL(k_lines_msg, dim3(blocks_for(n)), dim3(BLOCK), 0, s, hm, n, guard);
}
void launch_lines_at_p(const Pair3Args& a, LineEntry* ev, hipStream_t s) {
  if (a.f_n)
    hipLaunchKernelGGL(k_lines_at_p, dim3(blocks_for(a.f_n)), dim3(BLOCK), 0, s, a.pk, a.pk_st, a.msg_idx, a.hm, a.f_n, ev);
}
template <int MODE>
static void pair3_launch(const Pair3Args& a, hipStream_t s) {
  if (!a.n) return;
  unsigned grid = (unsigned)((a.n + GROUPS_PER_WAVE - 1) / GROUPS_PER_WAVE);
  hipLaunchKernelGGL(k_pair3<MODE>, dim3(grid), dim3(64), 0, s, a);
}
void launch_pair3(const Pair3Args& a, hipStream_t s) { pair3_launch<P3_FULL>(a, s); }
void launch_pair3_ml(const Pair3Args& a, hipStream_t s) { pair3_launch<P3_ML>(a, s); }
void launch_pair3_fin(const Pair3Args& a, hipStream_t s) { pair3_launch<P3_FIN>(a, s); }
void launch_pair3_prod(const Pair3Args& a, hipStream_t s) { pair3_launch<P3_PROD>(a, s); }
void launch_pair3_mml(const Pair3Args& a, hipStream_t s) { pair3_launch<P3_MML>(a, s); }
void launch_pair3_mls(const Pair3Args& a, hipStream_t s) { pair3_launch<P3_MLS>(a, s); }

}  // namespace hb
