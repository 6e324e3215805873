"""Paths the round-5 review found unguarded, -m gpu through the C ABI.

* A verification group whose items name different messages, inside a slot that defers its
  messages' Miller lines (distinct per-validator messages, the slot-wide check): the group is not
  READY, so its items are checked one by one against the unevaluated lines -- which the slot must
  then compute although the slot-wide check passed (hipbls.hip k_slot_verdict sets the flag
  k_lines_msg waits on).
* A large host-buffer Verify split into chunks (verify_large) whose chunks fall below the batched
  final exponentiation's group count while the whole call is above it: each chunk decides its
  deferred lines from its own size (no "deferred Miller lines need the batched final
  exponentiation" error).
* The decompressed-signature cache under concurrent callers: puts run beside the next calls and
  gets never wait for a Verify still in its pipeline -- every status and aggregate stays exact, and
  a single Verify's latency beside a large Verify is reported.
"""
import ctypes
import os
import sys
import threading
import time

import numpy as np
import pytest

from charon_amd import _lib
from charon_amd._lib import NOT_VERIFIED, OK

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _p(x):
    if x is None:
        return None
    if isinstance(x, np.ndarray):
        return ctypes.c_void_p(x.ctypes.data)
    return ctypes.c_void_p(x.data_ptr())


def _chk(L, rc):
    assert rc == 0, L.hbls_last_error().decode()


@pytest.fixture(scope="module")
def L(hipbls):
    return _lib.load_library()


def _sign_one(L, sk32, msg32):
    out = np.zeros(96, dtype=np.uint8)
    st = np.zeros(1, dtype=np.uint8)
    off = np.zeros(1, dtype=np.uint64)
    ln = np.full(1, 32, dtype=np.uint32)
    _chk(L, L.hbls_sign_batch(_p(np.ascontiguousarray(sk32)), _p(np.ascontiguousarray(msg32)), _p(off), _p(ln), 1,
                              _p(out), _p(st)))
    assert st[0] == 0
    return out


def test_slot_inconsistent_group_with_deferred_lines(L, monkeypatch):
    import bench
    from test_gpu_configs import _run_slot
    wl = dict(validators=4096, n=4, t=3, distinct=True, n_msgs=0)
    d = dict(bench.setup_inputs(L, wl, wl["validators"], 0))
    V, n, NP = d["V"], d["n"], d["NP"]
    assert d["M"] == V  # one message per validator: the slot defers its lines
    outside = [p for p in range(n) if p not in set(bench.ta_share_positions(n, d["t"]))][0]
    msgs = d["msgs"].reshape(V, 32)
    midx = d["midx"].copy()
    sigs = d["sigs"].copy().reshape(NP, 96)
    exp = np.zeros(NP, dtype=np.uint8)
    # validator 5: one partial (outside the aggregated members) signed over validator 6's message
    # and naming it -- valid, but the group is inconsistent
    i = 5 * n + outside
    midx[i] = 6
    sigs[i] = _sign_one(L, d["sks"][32 * i:32 * i + 32], msgs[6])
    # validator 9: one partial naming validator 10's message, still signed over its own -- invalid
    j = 9 * n + outside
    midx[j] = 10
    exp[j] = NOT_VERIFIED
    d["midx"] = midx
    d["sigs"] = sigs.reshape(-1)
    monkeypatch.setenv("HBLS_STATS", "1")
    prev = L.hbls_slot_msm(1)  # the slot-wide check at this size
    L.hbls_slot_msm(1)  # (and a clean adaptive history)
    try:
        s0 = (ctypes.c_uint64 * 6)()
        assert L.hbls_stats(s0, 6) == 0
        vst, tst, ast, tout = _run_slot(L, d, sigs=d["sigs"])
        s1 = (ctypes.c_uint64 * 6)()
        assert L.hbls_stats(s1, 6) == 0
    finally:
        L.hbls_slot_msm(prev)
    tried, failed = s1[4] - s0[4], s1[5] - s0[5]
    assert tried == 1 and failed == 0, (tried, failed)  # the inconsistent groups are outside the check
    bad = np.nonzero(vst != exp)[0]
    assert len(bad) == 0, [(int(k), int(vst[k]), int(exp[k])) for k in bad[:10]]
    assert int((tst != OK).sum()) == 0 and int((ast != OK).sum()) == 0
    assert np.array_equal(tout, d["root_sigs"].reshape(V, 96))


@pytest.fixture(scope="module")
def large(L):
    """2^19 + partials over distinct per-validator messages: hbls_verify_batch takes verify_large
    (chunks over the host-call contexts) with deferred lines."""
    import bench
    wl = dict(validators=53_000, n=10, t=7, distinct=True, n_msgs=0)
    return bench.setup_inputs(L, wl, wl["validators"], 0)


def test_verify_large_chunks_below_fe_batch(L, large):
    d = large
    NP, V = d["NP"], d["V"]
    assert NP >= 1 << 19
    # the whole call's 53 000 groups take the batched final exponentiation, each chunk's ~26 500 not
    prev = L.hbls_fe_batch(40_000)
    try:
        st = np.full(NP, 255, dtype=np.uint8)
        _chk(L, L.hbls_verify_batch(_p(d["pks"]), _p(d["sigs"]), _p(d["item_msgs"]), _p(d["item_off"]),
                                    _p(d["item_len"]), NP, _p(st)))
        assert int((st != OK).sum()) == 0
        # and with one invalid partial: exact
        sigs = d["sigs"].copy().reshape(NP, 96)
        k = 12_345
        sigs[k] = sigs[k + 1]
        _chk(L, L.hbls_verify_batch(_p(d["pks"]), _p(sigs.reshape(-1)), _p(d["item_msgs"]), _p(d["item_off"]),
                                    _p(d["item_len"]), NP, _p(st)))
        assert [int(x) for x in np.nonzero(st != OK)[0]] == [k] and st[k] == NOT_VERIFIED
    finally:
        L.hbls_fe_batch(prev)
    assert V == 53_000


def test_sig_cache_concurrent_callers(L, large):
    """A large Verify (signature-cache puts), ThresholdAggregate batches of the same partials
    (cache gets) and single Verifies from three threads at once, several rounds: every status and
    aggregate exact.  The single Verify's latency beside the large calls is printed (a put no longer
    sits on another call's stream, so a small call does not wait for the large one)."""
    d = large
    NP, V = d["NP"], d["V"]
    errors = []
    lat = []
    stop = threading.Event()

    def verify_large():
        st = np.zeros(NP, dtype=np.uint8)
        for _ in range(3):
            rc = L.hbls_verify_batch(_p(d["pks"]), _p(d["sigs"]), _p(d["item_msgs"]), _p(d["item_off"]),
                                     _p(d["item_len"]), NP, _p(st))
            if rc != 0 or (st != OK).any():
                errors.append(("verify", rc, int((st != OK).sum())))

    def aggregate():
        out = np.zeros(V * 96, dtype=np.uint8)
        st = np.zeros(V, dtype=np.uint8)
        for _ in range(3):
            rc = L.hbls_threshold_aggregate_batch(_p(d["ta_sigs"]), _p(d["ta_idx"]), _p(d["grp_off"]), V, _p(out),
                                                  _p(st))
            if rc != 0 or (st != OK).any() or not np.array_equal(out, d["root_sigs"]):
                errors.append(("aggregate", rc, int((st != OK).sum())))

    def single():
        st = np.zeros(1, dtype=np.uint8)
        off0 = np.zeros(1, dtype=np.uint64)
        len32 = np.full(1, 32, dtype=np.uint32)
        k = 0
        while not stop.is_set():
            i = (k * 7919) % NP
            t0 = time.perf_counter()
            rc = L.hbls_verify_batch(_p(d["pks"][48 * i:]), _p(d["sigs"][96 * i:]), _p(d["item_msgs"][32 * i:]),
                                     _p(off0), _p(len32), 1, _p(st))
            lat.append(time.perf_counter() - t0)
            if rc != 0 or st[0] != OK:
                errors.append(("single", rc, int(st[0])))
            k += 1

    ths = [threading.Thread(target=f) for f in (verify_large, aggregate)]
    ts = threading.Thread(target=single)
    ts.start()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    stop.set()
    ts.join()
    assert not errors, errors[:5]
    assert lat
    print(f"single Verify beside large calls: {len(lat)} calls, median {1e3 * sorted(lat)[len(lat) // 2]:.2f} ms, "
          f"max {1e3 * max(lat):.2f} ms")
