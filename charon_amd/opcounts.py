"""Algorithmic work per kernel unit for the roofline.

All work is counted in Fp Montgomery products (squarings counted as products): the building
blocks below are counted by the op-counting host build of the kernels' own arithmetic
(tests/native/hostcheck.cpp hc_count_blocks) and re-derived by tests/test_opcount.py.  One Fp
product is MAC_PER_FPMUL = 2*12*12 + 12 = 300 32x32->64-bit multiply-adds (textbook 12-limb
CIOS), the unit of the peak.

PEAK_MAD_TOPS: v_mad_u64_u32 lane-ops/s on MI355X, measured by tools/microbench/int_rates.hip at
16 waves/CU with 2 ms kernels (profiles/r05b_int_rates_traced.txt: 32.654 Tops/s, event-timed) and
pinned by counters (profiles/r05b_peak_from_counters.json: SQ_INSTS_VALU x 64 over the traced
duration 32.739 T, 262 185 VALU instructions per wave for the 262 144 issued; GRBM_GUI_ACTIVE / 8
XCDs: 2365 MHz).  That is 53.9 lane-ops per clock per CU, 84 % of the 64 a wave64 instruction per
SIMD per 4 clocks allows.  PEAK_MAD_TOPS_NOMINAL: the 64 lane-ops/clk/CU x 256 CUs at the nominal
2.4 GHz.  (Round 1's 29.944 T came from 0.5 ms kernels that ran at ~2.16 GHz: the same 53.9 per
clock at a lower clock.)

Per kernel two counts: `alg` is the textbook tower-arithmetic work of the unit (what a one-lane
implementation of the same algorithm executes); `exec` is what the kernel executes (e.g. the
three-lane pairing evaluates every H(m) line in all three lanes and inverts in all three).
"""

MAC_PER_FPMUL = 2 * 12 * 12 + 12
PEAK_MAD_TOPS = 32.654
PEAK_MAD_TOPS_NOMINAL = 39.322
PEAK_CLOCK_MHZ = 2365  # the effective clock PEAK_MAD_TOPS was measured at
PEAK_SOURCE = "profiles/r05b_peak_from_counters.json"

# hc_count_blocks, in its order
BLOCK_NAMES = ("f12_sqr", "f12_mul_line", "final_exp", "fp_inv", "g1_dec", "g2_dec", "rlc_g1", "rlc_g2",
               "jac_add_g1", "jac_add_g2", "to_aff_g1", "to_aff_g2", "lines_eval", "lines_uneval", "jac_dbl_g2",
               "jac_add_aff_g2", "cyclo_sqr", "f12_mul", "g2_compress", "jac_add_aff_g1", "jac_dbl_g1")
# fp_inv: the inversion by divsteps (fp.h, round 4) runs no Montgomery product but its final
# conversion to Montgomery form (463 as a^(p-2) before); its ~20 000 32-bit operations per inversion
# count as overhead, not as algorithmic work
BLOCKS = dict(zip(BLOCK_NAMES, (36, 39, 7679, 1, 1492, 2127, 732, 1880, 16, 43, 5, 16, 1843, 1571, 16, 29, 18,
                                54, 4, 11, 7)))

G2_DEC_LAZY_EXTRA = 5  # ec28.h g2l_madd / g2l_add against ec.h jac_add_aff / jac_add (5 x 1; g2l_dbl is the textbook 2M + 5S since round 4)
N_LINES = 68      # Miller-loop lines (63 doublings + 5 additions)
N_SQR = 62        # Fp12 squarings of the Miller loop
LINE_PRODUCTS = 2 * N_LINES  # two pairs per check

# expand_message_xmd -> 2 inversion-free SSWU + 3-isogeny maps (2 exponentiations each; 6188 with
# the inversion, 3 exponentiations) -> cofactor -> affine (5374 with the inversion as a^(p-2))
HASH_TO_G2 = 4912


def _pair3_exec_per_lane(b=BLOCKS):
    """Executed Fp products per lane of pair3.h's final exponentiation (3 lanes per pairing)."""
    f4_mul, f4_sqr, g_mul, frob = 9, 6, 18, 6
    g_inv = f4_sqr + f4_mul + f4_mul + 4 + (b["fp_inv"] + 4) + 6 + f4_mul
    pow_x = 63 * 6 + 5 * g_mul
    return (g_mul + g_inv) + (frob + g_mul) + 5 * pow_x + 2 * g_mul + (frob + g_mul) + (frob + 2 * g_mul) + \
        (6 + 2 * g_mul)


def pair3(b=BLOCKS):
    """k_pair3, per pairing check (Miller loop over precomputed lines + final exponentiation)."""
    alg = N_SQR * b["f12_sqr"] + LINE_PRODUCTS * b["f12_mul_line"] + N_LINES * 4 + b["final_exp"]
    exe = N_SQR * 36 + LINE_PRODUCTS * 45 + N_LINES * 12 + 3 * _pair3_exec_per_lane(b)
    return alg, exe


FE_BATCH = 64    # groups per batched final exponentiation (layout.h)


def pair3_ml(b=BLOCKS):
    """k_pair3_ml, per verification group: the Miller loop of (P, H(m)) alone, stored."""
    alg = N_SQR * b["f12_sqr"] + N_LINES * b["f12_mul_line"] + N_LINES * 4
    exe = N_SQR * 36 + N_LINES * 45 + N_LINES * 12
    return alg, exe


MML_PAIRS = 4    # pairs per multi-Miller loop of the slot-wide check (layout.h)


def pair3_mml(b=BLOCKS, pairs=MML_PAIRS):
    """k_pair3_mml per verification group: its 68 line products (the lines come evaluated at P,
    k_mml_eval) in a Miller loop whose 62 squarings `pairs` groups share."""
    alg = N_LINES * b["f12_mul_line"] + N_SQR * b["f12_sqr"] / pairs
    exe = N_LINES * 45 + N_SQR * 36 / pairs
    return alg, exe


def mml_eval(b=BLOCKS):
    """k_mml_eval per verification group: its 68 lines evaluated at P once (two Fp2 x Fp products
    each), where the three lanes of a multi-Miller loop group each repeated them."""
    return (N_LINES * 4,) * 2


def mml_pairs(groups, n_cu=256, groups_per_wave=21):
    """The library's pairs per multi-Miller loop (hipbls.hip verify_pipeline): enough that the loops
    fit one round of waves, one wave per SIMD (4 per CU)."""
    return min(16, max(1, -(-groups // (groups_per_wave * 4 * n_cu))))


def pair3_fin(b=BLOCKS, batch=FE_BATCH, lines=True):
    """k_pair3_fin, per final exponentiation: the Miller loop of (-g1, sum S) (unless lines=False:
    k_pair3_mls computed it beside the product tree), times `batch` stored values, exponentiated."""
    ml = (N_SQR * b["f12_sqr"] + N_LINES * b["f12_mul_line"], N_SQR * 36 + N_LINES * 45) if lines else (0, 0)
    alg = ml[0] + batch * b["f12_mul"] + b["final_exp"]
    exe = ml[1] + batch * 54 + 3 * _pair3_exec_per_lane(b)
    return alg, exe


def pair3_mls(b=BLOCKS):
    """k_pair3_mls, per final exponentiation: the Miller loop of (-g1, S) alone, stored."""
    return N_SQR * b["f12_sqr"] + N_LINES * b["f12_mul_line"], N_SQR * 36 + N_LINES * 45


PROD_FAN = 8     # fan-in of the product trees in front of a final exponentiation (layout.h)


def prod_tree_inputs(n, fan=PROD_FAN):
    """Stored values multiplied by a product tree of fan-in `fan` down to one value."""
    tot = 0
    while True:
        tot += n
        n = -(-n // fan)
        if n <= 1:
            return tot


RLC_CHUNK = 16   # items per lane of k_rlc_msm (layout.h)
TA_CHUNK = 8     # members per lane of k_ta_msm (layout.h)


def rlc_msm(b=BLOCKS, chunk=1, sides=3):
    """k_rlc_msm per item of a chunk of `chunk` items: the ladder points (phi + one mixed addition
    per side; affine on the G1 side), 32 shared doublings per chunk, 32 additions per item.  sides: 1 the public-key side
    only (the slot-wide check takes the signature side as one MSM), 3 both."""
    # G1: P + phi(P) made affine with one inversion per chunk (3 products into and out of the
    # running product, 1/Z^2, 1/Z^3, x, y), then 32 mixed additions
    g1 = 1 + b["jac_add_aff_g1"] + 3 + 4 + b["fp_inv"] / chunk + 32 * b["jac_add_aff_g1"] + 32 * b["jac_dbl_g1"] / chunk
    # G2 likewise: S + (-psi^2 S) affine with one Fp2 inversion per chunk (products into and out of
    # the running product 3 x 3, then 1/Z^2, 1/Z^3, x, y: 2 + 3 x 3), 32 mixed additions
    g2 = 6 + b["jac_add_aff_g2"] + 9 + 11 + (b["fp_inv"] + 6) / chunk + 32 * b["jac_add_aff_g2"] + \
        32 * b["jac_dbl_g2"] / chunk
    return g1 + (g2 if sides & 2 else 0)


# The slot-wide check's multi-scalar multiplication of the signature side (msm.hip): two windows of
# 16 bits over the two 32-bit halves of every coefficient, i.e. 4 bucket entries per item.
MSM_C, MSM_WINDOWS, MSM_CHUNK = 16, 2, 4
MSM_KEYS = MSM_WINDOWS << MSM_C
MSM_PARTS = MSM_KEYS // MSM_CHUNK
MSM_ENTRIES_PER_ITEM = 2 * MSM_WINDOWS


def msm_bucket(b=BLOCKS):
    """k_msm_bucket per entry: one mixed G2 addition; half the entries first map the point through
    -psi^2 (two Fp2-by-Fp products)."""
    return b["jac_add_aff_g2"] + 2


def msm_reduce(b=BLOCKS):
    """k_msm_reduce per chunk of MSM_CHUNK buckets: running sums (2 additions per bucket), one
    16-bit multiple (16 doublings, 16 additions), the window shift (16 doublings for window 1)."""
    return 2 * MSM_CHUNK * b["jac_add_g2"] + 16 * (b["jac_dbl_g2"] + b["jac_add_g2"]) + \
        16 * b["jac_dbl_g2"] * (MSM_WINDOWS - 1) / MSM_WINDOWS


def ta_msm(b=BLOCKS, chunk=1):
    """k_ta_table + k_ta_msm per member of a chunk of `chunk` members: the 15-entry subset table,
    64 shared doublings per chunk, 64 additions per member."""
    return 18 + 11 * b["jac_add_aff_g2"] + 64 * b["jac_add_g2"] + 64 * b["jac_dbl_g2"] / chunk


R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
X_ABS = 0xD201000000010000


def _naf4(v):
    """Signed width-4 NAF digits of v (least significant first), as k_ta_straus builds them."""
    out = []
    while v:
        d = 0
        if v & 1:
            d = v & 15
            if d >= 8:
                d -= 16
            v -= d
        out.append(d)
        v >>= 1
    return out


def ta_uniform(ids, b=BLOCKS):
    """k_ta_straus per member when a wave's Lagrange digits agree (every validator aggregates the
    share indices `ids`): the odd-multiple table (a doubling, three additions, the psi images),
    then top + 1 doublings and one addition per nonzero NAF digit of the four base-|x| digits of
    lambda_j(0).  Returns the mean over the members."""
    tot = 0
    for i in ids:
        lam = 1
        for j in ids:
            if j != i:
                lam = lam * j % R_ORDER * pow(j - i, -1, R_ORDER) % R_ORDER
        digits = []
        for _ in range(4):
            digits.append(lam % X_ABS)
            lam //= X_ABS
        nafs = [_naf4(a) for a in digits]
        top = max((len(n) for n in nafs), default=1)
        adds = sum(1 for n in nafs for d in n if d)
        table = b["jac_dbl_g2"] + b["jac_add_aff_g2"] + 2 * b["jac_add_g2"] + 4 * 24
        tot += table + top * b["jac_dbl_g2"] + adds * b["jac_add_g2"]
    return tot / len(ids)


def ta_joint(ids, chunk, b=BLOCKS):
    """k_ta_joint (threshold.hip) per member: a lane per chunk of `chunk` members of a validator
    aggregating the share indices `ids`; per member its affine odd-multiple table (one batched
    inversion per chunk), per chunk ONE schedule of top + 1 doublings (top over the chunk's
    members), one mixed addition per nonzero NAF digit."""
    lams = []
    for i in ids:
        lam = 1
        for j in ids:
            if j != i:
                lam = lam * j % R_ORDER * pow(j - i, -1, R_ORDER) % R_ORDER
        lams.append(lam)
    # per member: 2P, 3P, 5P, 7P; 3 products into the running product of Z; back: 2 products for
    # 1/Z, then 1/Z^2, 1/Z^3 and x, y (Fp2: sqr 2, mul 3 Fp products) for 3 points; psi images of
    # the 4 affine points (3 images x 2 Fp2 products); per chunk one Fp2 inversion
    table = b["jac_dbl_g2"] + b["jac_add_aff_g2"] + 2 * b["jac_add_g2"] + 3 * 3 + 3 * (2 * 3 + 2 + 3 * 3) + 4 * 18
    tot = 0
    for c0 in range(0, len(ids), chunk):
        top, adds = 0, 0
        for lam in lams[c0:c0 + chunk]:
            for _ in range(4):
                n = _naf4(lam % X_ABS)
                lam //= X_ABS
                adds += sum(1 for d in n if d)
                top = max(top, len(n))
            tot += table
        tot += b["fp_inv"] + 6 + top * b["jac_dbl_g2"] + adds * b["jac_add_aff_g2"]
    return tot / len(ids)


def ta_small_split(ids):
    """ta_small.h restated: (c_j, s) with lambda_j(0) = s c_j mod r and small integers c_j, or None
    where the library refuses the split (the per-member ladders run)."""
    from math import gcd
    t = len(ids)
    if t < 2 or t > 16 or any(x == 0 or abs(x) >= 2 ** 31 for x in ids) or len(set(ids)) != t:
        return None
    E = []
    for j in ids:
        e = j
        for m in ids:
            if m != j:
                e *= m - j
        E.append(e)
    L = 1
    for e in E:
        L = L // gcd(L, abs(e)) * abs(e)
    if L >= 2 ** 63 or any(abs(e) >= 2 ** 63 for e in E):
        return None
    P = 1
    for x in ids:
        P = P * x % R_ORDER
    return [L // e for e in E], P * pow(L, -1, R_ORDER) % R_ORDER


def _naf2(v):
    out = []
    while v:
        d = 0
        if v & 1:
            d = -1 if v & 2 else 1
            v -= d
        out.append(d)
        v >>= 1
    return out


def ta_small(ids, b=BLOCKS):
    """k_ta_small + k_ta_stab + k_ta_sladder (threshold.hip) per VALIDATOR aggregating the share
    indices `ids` through the small-scalar split: the joint signed-binary ladder over the c_j
    (shared doublings, one mixed addition per nonzero digit), the affine odd-multiple tables of Q
    (a doubling, three additions, one Fp2 inversion: 4 x 3 products into the running product, 17
    per point back out, the psi images 3 x 6 per point), then [s] Q by the width-4 NAF schedule of
    the four base-|x| digits of s.  None if the split is refused."""
    sp = ta_small_split(ids)
    if sp is None:
        return None
    c, s = sp
    nafs = [_naf2(abs(x)) for x in c]
    top = max(len(n) for n in nafs)
    adds = sum(1 for n in nafs for d in n if d)
    small = top * b["jac_dbl_g2"] + adds * b["jac_add_aff_g2"]
    table = b["jac_dbl_g2"] + 3 * b["jac_add_g2"] + b["fp_inv"] + 6 + 4 * 3 + 4 * 17 + 4 * 18
    digits = []
    for _ in range(4):
        digits.append(s % X_ABS)
        s //= X_ABS
    nafs = [_naf4(a) for a in digits]
    top4 = max((len(n) for n in nafs), default=1)
    adds4 = sum(1 for n in nafs for d in n if d)
    return small + table + top4 * b["jac_dbl_g2"] + adds4 * b["jac_add_aff_g2"]


def ta_joint_chunk(t, n_partials, knob=0, lanes=98304):
    """The library's choice of members per lane (hipbls.hip ta_tail): 0/1 = one ladder per member."""
    c = knob if knob else n_partials // lanes
    c = min(c, t, 8)
    return c if c > 1 else 0


def per_unit(b=BLOCKS, group_size=1, t=1):
    """{kernel: (alg, exec)} Fp products per unit (unit named in UNITS)."""
    p = pair3(b)
    k = group_size
    prep = (b["lines_eval"] if k == 1 else
            (k - 1) * (b["jac_add_g1"] + b["jac_add_g2"]) + b["to_aff_g1"] + b["to_aff_g2"] + b["lines_eval"])
    gsum = t * b["jac_add_g2"] + b["to_aff_g2"] + b["g2_compress"]
    out = {
        "k_pair3": p, "k_pair3_fallback": p,
        "k_dec_pk": (b["g1_dec"],) * 2,
        # the lazy-limb ladder (ec28.h) spends one product more per doubling than dbl-2009-l's
        # 2M + 5S (D = 4XB as a product): 63 + 5 executed, the textbook 2M + 5S counted as alg
        "k_dec_sig_pt": (b["g2_dec"] - G2_DEC_LAZY_EXTRA, b["g2_dec"]),
        # one chunk per verification group of <= RLC_CHUNK items (the slot's groups of n + 1)
        "k_rlc": (rlc_msm(b, min(group_size, RLC_CHUNK)),) * 2,
        "k_group_prep": (prep,) * 2,
        "k_fb_lines": (b["lines_eval"],) * 2,
        "k_ta_straus": (ta_msm(b, 1),) * 2,  # one ladder per member
        "k_group_sum": (gsum,) * 2,
        # the two cofactor ladders in lazy limbs (ec28.h): one product more per doubling / addition
        "k_hash_to_g2": (HASH_TO_G2, HASH_TO_G2 + 2 * G2_DEC_LAZY_EXTRA),
        "k_lines_msg": (b["lines_uneval"],) * 2,
        # VerifyAggregate at scale (vbatch.hip): per key one mixed addition in pass 1 (later passes
        # add 1/32 as many Jacobian partials), per group the affine sum and the signature's lines
        "k_seg_sum": (b["jac_add_aff_g1"],) * 2,
        "k_va_point": (b["to_aff_g1"],) * 2,
        "k_sig_lines": (b["lines_eval"],) * 2,
        # batched final exponentiation (vgroup.hip): per group the sums, the affine key, one share
        # of the batch sum (executed: the six-level butterfly in every lane) and the stored loop;
        # per batch the lines of the summed signature side and the shared exponentiation
        "k_group_prep_b": ((k - 1) * (b["jac_add_g1"] + b["jac_add_g2"]) + b["to_aff_g1"] + b["jac_add_g2"],
                           (k - 1) * (b["jac_add_g1"] + b["jac_add_g2"]) + b["to_aff_g1"] + 6 * b["jac_add_g2"]),
        "k_pair3_ml": pair3_ml(b),
        "k_pair3_fin": pair3_fin(b, batch=2, lines=False),
        "k_pair3_mls": pair3_mls(b),
        "k_slines": (b["to_aff_g2"] + b["lines_eval"],) * 2,
        # slot-wide check (msm.hip): per group the key sum alone; the product tree of the stored
        # loops (one Fp12 product per stored value); the MSM kernels per entry / chunk / point
        "k_group_prep_p": ((k - 1) * b["jac_add_g1"] + b["to_aff_g1"],) * 2,
        "k_pair3_prod": (b["f12_mul"], 3 * 18),
        "k_pair3_mml": pair3_mml(b),
        "k_mml_eval": mml_eval(b),
        # distinct-message slots (round 5): the chain of H(m_g) evaluated at P_g inside it
        "k_lines_at_p": (b["lines_uneval"] + mml_eval(b)[0],) * 2,
        "k_msm_bucket": (msm_bucket(b),) * 2,
        "k_msm_reduce": (msm_reduce(b),) * 2,
        "k_msm_sum": (b["jac_add_g2"],) * 2,
    }
    return out


UNITS = {"k_pair3": "pairing check", "k_pair3_fallback": "pairing check", "k_dec_pk": "public key",
         "k_dec_sig_pt": "signature", "k_rlc": "partial", "k_group_prep": "verification group",
         "k_fb_lines": "partial", "k_ta_straus": "aggregation member", "k_group_sum": "aggregation group",
         "k_hash_to_g2": "message", "k_lines_msg": "message", "k_seg_sum": "public key (pass 1)",
         "k_va_point": "aggregation group", "k_sig_lines": "signature", "k_group_prep_b": "verification group",
         "k_pair3_ml": "verification group", "k_pair3_fin": "final exponentiation",
         "k_slines": "batch of 64 groups", "k_group_prep_p": "verification group",
         "k_pair3_prod": "stored Miller loop", "k_pair3_mml": "verification group", "k_msm_bucket": "bucket entry", "k_msm_reduce": "chunk of 16 buckets",
         "k_msm_sum": "point", "k_mml_eval": "verification group", "k_lines_at_p": "verification group", "k_pair3_mls": "final exponentiation", "k_ta_small": "aggregation group (validator)"}

# SHA-256 compressions per attestation signing root (roots.hip: 8 two-block hashes)
SHA256_PER_ATTESTATION_ROOT = 16

# The herumi-equivalent per-item work of r01 (frozen): one Verify = G1 + G2 decompression with
# subgroup checks + a 2-pair Miller loop with line construction + final exponentiation, counted
# on the r01 algorithms.  The slot's effective rate is quoted against it.
FPMUL_PER_ITEM_R01 = {"verify": 29601, "hash_to_g2": 7813}
