"""First-error verification of an ordered set (hbls_verify_batch_first_error and
hbls_verify_device_first_error), -m gpu.

The reference's callers stop at the first failing partial of a set (core/parsigex/parsigex.go:93-98,
core/sigagg/sigagg.go:56-63, core/validatorapi/validatorapi.go:302-306).  The first-error mode
must report exactly the item the exact per-item statuses (hbls_verify_batch) name first, with
the same status, on the C5 mix (bench.corrupt: 1 % of the partials corrupted in fifths), on sets
whose every item is bad (undecodable, or decodable and wrong), on single bad items at chosen
positions and on clean sets -- through the slot-wide check, the per-batch check behind it (the
adaptive state after a failing call), distinct per-validator messages with deferred lines, and the
device entry point.
"""
import ctypes
import os
import random
import sys

import numpy as np
import pytest

from charon_amd import _lib
from charon_amd._lib import BAD_SIGNATURE, NOT_VERIFIED, OK, UNCHECKED

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


def _exact(L, d, sigs):
    st = np.full(d["NP"], 255, dtype=np.uint8)
    _chk(L, L.hbls_verify_batch(_p(d["pks"]), _p(sigs), _p(d["item_msgs"]), _p(d["item_off"]), _p(d["item_len"]),
                                d["NP"], _p(st)))
    return st


def _first(L, d, sigs):
    NP = d["NP"]
    first = ctypes.c_int64(-2)
    fst = ctypes.c_uint8(255)
    st = np.full(NP, 255, dtype=np.uint8)
    _chk(L, L.hbls_verify_batch_first_error(_p(d["pks"]), _p(sigs), _p(d["item_msgs"]), _p(d["item_off"]),
                                            _p(d["item_len"]), NP, ctypes.byref(first), ctypes.byref(fst), _p(st)))
    return int(first.value), int(fst.value), st


def _check_against_exact(L, d, sigs, label):
    exact = _exact(L, d, sigs)
    bad = np.nonzero(exact != OK)[0]
    for rep in range(2):  # the second call after a failing one: the adaptive per-batch path
        f, fs, st = _first(L, d, sigs)
        if len(bad) == 0:
            assert f == -1 and fs == OK, (label, f, fs)
            assert (st == OK).all(), label
            continue
        assert f == int(bad[0]), (label, rep, f, int(bad[0]))
        assert fs == int(exact[f]), (label, rep, fs, int(exact[f]))
        assert (st[:f] == OK).all(), label
        after = st[f + 1:]
        # after the first failure: the exact status or UNCHECKED, nothing else
        assert ((after == exact[f + 1:]) | (after == UNCHECKED)).all(), label
    return exact


@pytest.fixture(scope="module", params=["c5mix", "distinct"])
def cluster(L, request):
    import bench
    if request.param == "c5mix":  # 64 shared messages, runs of a validator's 7 partials
        wl = dict(validators=12_000, n=7, t=5, distinct=False, n_msgs=64)
    else:  # one message per validator (deferred lines)
        wl = dict(validators=4_000, n=10, t=7, distinct=True, n_msgs=0)
    return bench.setup_inputs(L, wl, wl["validators"], 0)


def test_first_error_c5_mix(L, cluster):
    import bench
    d = dict(cluster)
    d["sigs"] = cluster["sigs"].copy()
    bench.corrupt(L, d, 0.01, seed=17)
    exact = _check_against_exact(L, d, d["sigs"], "c5")
    assert set(np.unique(exact).tolist()) == {OK, BAD_SIGNATURE, NOT_VERIFIED}


def test_first_error_clean_and_single_bad(L, cluster):
    d = cluster
    NP = d["NP"]
    _check_against_exact(L, d, d["sigs"], "clean")
    rng = random.Random(5)
    sig = d["sigs"].reshape(NP, 96)
    for pos in (0, NP // 3, NP - 1, rng.randrange(NP)):
        s2 = sig.copy()
        s2[pos] = sig[(pos + 1) % NP]  # another partial: decodable, NOT_VERIFIED
        exact = _check_against_exact(L, d, s2.reshape(-1), f"one bad at {pos}")
        assert [int(x) for x in np.nonzero(exact != OK)[0]] == [pos]


def test_first_error_all_bad(L, cluster):
    d = cluster
    NP = d["NP"]
    sig = d["sigs"].reshape(NP, 96)
    rolled = np.roll(sig, 1, axis=0)  # every item carries another item's signature: all NOT_VERIFIED
    exact = _check_against_exact(L, d, rolled.reshape(-1).copy(), "all decodable wrong")
    assert (exact == NOT_VERIFIED).all()
    junk = np.zeros_like(sig)
    junk[:, 0] = 0x1F  # no compression flag: undecodable
    exact = _check_against_exact(L, d, junk.reshape(-1).copy(), "all undecodable")
    assert (exact == BAD_SIGNATURE).all()
    # the first half clean, every item of the second half wrong
    half = sig.copy()
    half[NP // 2:] = rolled[NP // 2:]
    exact = _check_against_exact(L, d, half.reshape(-1).copy(), "second half wrong")
    assert int(np.nonzero(exact != OK)[0][0]) == NP // 2


def test_first_error_device_entry(L, cluster):
    """hbls_verify_device_first_error on the same set: the first index in a device word."""
    import bench
    import torch
    d = dict(cluster)
    d["sigs"] = cluster["sigs"].copy()
    bench.corrupt(L, d, 0.005, seed=23)
    exact = _exact(L, d, d["sigs"])
    dev = torch.device("cuda", 0)
    up = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    NP, M, V = d["NP"], d["M"], d["V"]
    g_msg, g_off, g_len = up(d["msgs"]), up(d["moff"].view(np.int64)), up(d["mlen"].view(np.int32))
    g_pk, g_sig, g_idx, g_voff = up(d["pks"]), up(d["sigs"]), up(d["midx"].view(np.int32)), up(d["vgrp_off"].view(np.int32))
    hm = torch.zeros(M * L.hbls_hm_entry_bytes(), dtype=torch.uint8, device=dev)
    st = torch.full((NP,), 255, dtype=torch.uint8, device=dev)
    first = torch.zeros(1, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(device=dev)
    sp = ctypes.c_void_p(s.cuda_stream)
    _chk(L, L.hbls_hash_to_g2_device(_p(g_msg), _p(g_off), _p(g_len), M, _p(hm), sp))
    _chk(L, L.hbls_verify_device_first_error(_p(g_pk), _p(g_sig), _p(g_idx), _p(hm), NP, _p(g_voff), V, _p(st),
                                             _p(first), sp))
    s.synchronize()
    f = int(first.cpu().numpy().view(np.uint32)[0])
    bad = np.nonzero(exact != OK)[0]
    assert f == int(bad[0])
    stv = st.cpu().numpy()
    assert stv[f] == exact[f] and (stv[:f] == OK).all()
    assert ((stv[f + 1:] == exact[f + 1:]) | (stv[f + 1:] == UNCHECKED)).all()
    # far fewer items resolved alone than the exact call's failing groups hold
    assert (stv == UNCHECKED).sum() > 0


def test_parsigex_mirror_uses_first_error(hipbls):
    """charon_amd.callers.parsigex_verify_set over the library: the first bad partial of a set
    raises the reference's error chain (parsigex.go:96, signing.go / herumi.go:300)."""
    from charon_amd import callers
    from charon_amd.tbls import TblsError
    import hashlib
    sks = [hashlib.sha256(b"first error key %d" % k).digest()[:31].rjust(32, b"\0") for k in range(3)]
    pks = [hipbls.secret_to_public_key(sk) for sk in sks]
    roots = [bytes([k]) * 32 for k in range(3)]
    sigs = [hipbls.sign(sk, r) for sk, r in zip(sks, roots)]
    dvs = [bytes([0xA0 + k]) * 48 for k in range(3)]
    shares = {dv: {1: pk} for dv, pk in zip(dvs, pks)}
    good = [(dv, callers.ParSig(1, r, s)) for dv, r, s in zip(dvs, roots, sigs)]
    callers.parsigex_verify_set(hipbls, shares, good)
    bad = list(good)
    bad[1] = (dvs[1], callers.ParSig(1, roots[1], sigs[2]))
    with pytest.raises(TblsError, match="invalid partial signature: invalid signature: signature not verified"):
        callers.parsigex_verify_set(hipbls, shares, bad)
