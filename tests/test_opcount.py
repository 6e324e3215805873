"""The algorithmic work per kernel unit (charon_amd/opcounts.py) is what the
kernels' own arithmetic executes: re-count the building blocks with the op-counting host build of
the kernels' code (tests/native/hostcheck.cpp) on an oracle fixture, and the r01 per-item count
the slot's effective rate is quoted against."""
import ctypes

import pytest

from charon_amd import opcounts


@pytest.fixture(scope="module")
def hc():
    import os
    from charon_amd.build import build_hostcheck
    # HBLS_HOSTCHECK_LIB: another build of the harness (tests/test_sanitizers.py: ASan + UBSan)
    return ctypes.CDLL(os.environ.get("HBLS_HOSTCHECK_LIB") or build_hostcheck(verbose=False))


def _valid(fixtures):
    return {x["name"]: x for x in fixtures["verify"]}["valid_share_1"]


def test_block_counts(hc, fixtures):
    c = _valid(fixtures)
    out = (ctypes.c_ulonglong * 32)()
    assert hc.hc_count_blocks(bytes.fromhex(c["pk"]), bytes.fromhex(c["sig"]), out) == 0
    got = dict(zip(opcounts.BLOCK_NAMES, list(out)[:len(opcounts.BLOCK_NAMES)]))
    assert got == opcounts.BLOCKS


def test_pair3_counts():
    alg, exe = opcounts.pair3()
    # Miller loop over precomputed lines: 62 Fp12 squarings, 136 sparse line products, 68 line
    # evaluations at P (2 Fp2 x Fp products each), then the final exponentiation
    assert alg == 62 * 36 + 136 * 39 + 68 * 4 + 7679
    assert exe > alg  # the three-lane kernel repeats the evaluations and the inversion per lane


def test_verify_count_r01_not_exceeded(hc, fixtures):
    """The herumi-equivalent per-item count of r01 is an upper bound of today's per-item path."""
    c = _valid(fixtures)
    out = (ctypes.c_ulonglong * 5)()
    m = bytes.fromhex(c["msg"])
    assert hc.hc_count_verify(bytes.fromhex(c["pk"]), m, len(m), bytes.fromhex(c["sig"]), out) == 0
    assert out[0] <= opcounts.FPMUL_PER_ITEM_R01["verify"]
    assert out[1] == opcounts.HASH_TO_G2


def test_batched_verify_work_below_per_item():
    """Per partial of a 10-partial group, the batched path's work is far below one pairing per
    partial (the point of the random linear combination)."""
    u = opcounts.per_unit(group_size=11, t=7)
    per_partial = (u["k_dec_pk"][0] + u["k_dec_sig_pt"][0] + u["k_rlc"][0] +
                   (u["k_group_prep"][0] + u["k_pair3"][0]) / 10)
    assert per_partial < 0.5 * opcounts.FPMUL_PER_ITEM_R01["verify"]


def test_mac_per_fpmul():
    assert opcounts.MAC_PER_FPMUL == 300
