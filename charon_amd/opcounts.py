"""Frozen algorithmic work per unit for the roofline.

FPMUL_PER_ITEM: Fp Montgomery products (squarings counted as products) per item, counted by the
op-counting host build of the kernels' own arithmetic (tests/native/hostcheck.cpp, hc_count_*) on
the r01 algorithms and frozen here, so that later algorithmic savings show up as a higher
effective fraction; tests/test_opcount.py re-derives the r01 numbers.

MAC_PER_FPMUL: one 12-limb CIOS Montgomery product = 2*12*12 + 12 = 300 32x32->64 multiply-adds.
PEAK_MAD_TOPS: v_mad_u64_u32 lane-ops/s on MI355X, measured by tools/microbench/int_rates.hip
(profiles/r01_int_rates_microbench.txt, 16 waves/CU: 29.944 Tops/s).
"""

MAC_PER_FPMUL = 2 * 12 * 12 + 12
PEAK_MAD_TOPS = 29.944

# Executed Fp products of the current kernels' arithmetic (algorithmic savings since r01, e.g.
# cyclotomic squaring in the final exponentiation); tests/test_opcount.py re-counts these too.
EXECUTED_FPMUL_PER_ITEM = {
    "k_verify": 23913,
    # straight-line SSWU (three exponentiations per map; the r01 map took a divergent fourth or
    # fifth on the non-square branch)
    "k_hash_to_g2": 7217,
}

FPMUL_PER_ITEM = {
    # per partial: G1 decompress+subgroup 1665, G2 decompress+subgroup 2486, 2-pair Miller loop +
    # final exponentiation 25450
    "k_verify": 29601,
    # the pairing part alone (k_pair3: 2-pair Miller loop + final exponentiation)
    "k_pair3": 25450,
    # per distinct 32-byte message: expand_message_xmd -> 2 SSWU -> 3-isogeny -> cofactor -> affine
    "k_hash_to_g2": 7813,
    # per validator of the bench's ThresholdAggregate (share indices {1,2,3}: lambda = 3, -3, 1;
    # decompress+subgroup + 255-bit double-and-add per partial; 428 Fr products each on top)
    "k_group_member_t3_123": 6595 + 11264 + 6566,
}
