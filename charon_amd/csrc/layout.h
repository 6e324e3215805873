// Device-side storage formats shared by the two translation units of libhipbls.so
// (hipbls.hip: host runtime + one-lane kernels; pipeline.hip: the staged verify pipeline).
#pragma once
#include "ops.h"

namespace hb {

struct HmEntry {  // affine G2 point (Montgomery limbs) + infinity flag, 208 B
  Fp2 x, y;
  uint32_t inf;
  uint32_t pad[3];
};

struct G2JEntry {  // Jacobian G2 point, 288 B
  Fp2 X, Y, Z;
};

struct G1AEntry {  // affine G1 point, 112 B
  Fp x, y;
  uint32_t inf;
  uint32_t pad[3];
};

struct LineEntry {  // one Miller-loop line, 288 B: (a0, c1, c2) unevaluated or (a0, a1, b1)
  Fp2 a0, a1, b1;
};

// Per distinct message: H(m) and the 68 unevaluated lines of its Miller chain (pairing.h
// miller_dbl_c / miller_add_c), shared by every partial signed over that message.
struct MsgEntry {
  HmEntry h;
  LineEntry lines[N_LINES];
};

__device__ __forceinline__ G2A hm_load(const HmEntry& e) { return {e.x, e.y, e.inf != 0}; }

// ThresholdAggregate member status flags (threshold.hip -> k_group_sum)
enum : uint8_t { M_OK = 0, M_BAD_SIG = 1, M_BAD_IDX = 2 };

// base-|x| digits of a Lagrange coefficient (threshold.hip)
struct TaDigits {
  uint64_t a[4];
};

// Staged ThresholdAggregate (threshold.hip)
void launch_ta_lambda(const int64_t* idx, const uint32_t* grp_off, uint32_t n_groups, uint32_t n_partials, int mode,
                      TaDigits* dig, uint8_t* mstat, hipStream_t s);
size_t ta_table_bytes(uint32_t n_partials);
void launch_ta_straus(const HmEntry* pts, const TaDigits* dig, uint32_t n_partials, void* tab, G2JEntry* out,
                      hipStream_t s);

// Staged verify pipeline (pipeline.hip): kernel launches on caller-provided streams.
constexpr int GROUPS_PER_WAVE = 21;  // k_pair3: 3 lanes per partial, 21 partials per wave
void launch_hash_to_g2(const uint8_t* msgs, const uint64_t* off, const uint32_t* len, uint32_t n, MsgEntry* hm,
                       hipStream_t s);
void launch_lines_msg(MsgEntry* hm, uint32_t n, hipStream_t s);
void launch_dec_pk(const uint8_t* pks, uint32_t n, G1AEntry* out, uint8_t* st, hipStream_t s);
void launch_dec_sig_lines(const uint8_t* sigs, uint32_t n, uint8_t* inf, uint8_t* st, LineEntry* lines,
                          hipStream_t s);
void launch_pair3(const G1AEntry* pk, const uint8_t* pk_st, const uint8_t* sig_inf, const uint8_t* sig_st,
                  const uint32_t* msg_idx, const MsgEntry* hm, const LineEntry* sig_lines, uint32_t n,
                  uint8_t* status, hipStream_t s);

}  // namespace hb
