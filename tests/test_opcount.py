"""The frozen algorithmic work per item (charon_amd/opcounts.py) is what the r01
arithmetic actually executes: re-count it with the op-counting host build of the kernels' own code
(tests/native/hostcheck.cpp) on an oracle fixture."""
import ctypes

import pytest

from charon_amd import opcounts


@pytest.fixture(scope="module")
def hc():
    from charon_amd.build import build_hostcheck
    return ctypes.CDLL(build_hostcheck(verbose=False))


def test_verify_counts(hc, fixtures):
    c = {x["name"]: x for x in fixtures["verify"]}["valid_share_1"]
    out = (ctypes.c_ulonglong * 5)()
    m = bytes.fromhex(c["msg"])
    assert hc.hc_count_verify(bytes.fromhex(c["pk"]), m, len(m), bytes.fromhex(c["sig"]), out) == 0
    # the frozen r01 count is the roofline's work unit; the executed count may only go down
    assert out[0] == opcounts.EXECUTED_FPMUL_PER_ITEM["k_verify"]
    assert out[0] <= opcounts.FPMUL_PER_ITEM["k_verify"]
    assert out[1] == opcounts.EXECUTED_FPMUL_PER_ITEM["k_hash_to_g2"]
    assert out[1] <= opcounts.FPMUL_PER_ITEM["k_hash_to_g2"]


def test_threshold_aggregate_counts(hc, fixtures):
    c = {x["name"]: x for x in fixtures["threshold_aggregate"]}["t_of_n_123"]
    items = list(c["partials"].items())
    assert sorted(int(k) for k, _ in items) == [1, 2, 3]
    sigs = b"".join(bytes.fromhex(v) for _, v in items)
    idx = (ctypes.c_int64 * len(items))(*[int(k) for k, _ in items])
    total = 0
    for j in range(len(items)):
        out = (ctypes.c_ulonglong * 2)()
        assert hc.hc_count_ta_member(sigs, idx, len(items), j, out) == 0
        total += out[0]
    assert total == opcounts.FPMUL_PER_ITEM["k_group_member_t3_123"]


def test_mac_per_fpmul():
    assert opcounts.MAC_PER_FPMUL == 300
