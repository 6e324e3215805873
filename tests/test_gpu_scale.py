"""GPU parity at BASELINE sizes through the C ABI (-m gpu).

* The slot entry point (hbls_slot_device: hashing, batched verification, ThresholdAggregate over
  the verified partials, post-aggregate verification under the DV keys) on a C2-size cluster with
  the C5 adversarial mix: 1 % of the partials corrupted in equal fifths (random bytes, on-curve
  off-subgroup points, wrong message, wrong share index, infinity) plus a few undecodable public
  keys.  Expected statuses follow from the construction (reference semantics:
  core/parsigex/parsigex_test.go:285-289 random signature -> error, core/sigagg/sigagg_test.go
  wrong partials, validatorapi_test.go wrong message -> "signature not verified"), cross-checked
  on a sample by the oracle.
* VerifyAggregate with 512 public keys per message (sync committee, BASELINE configs[4]).
* Concurrent single-item callers (the library's coalescing queue) and a device entry point
  racing a host-buffer call on another stream (the workspaces are ordered by events).
"""
import ctypes
import os
import hashlib
import random
import threading

import numpy as np
import pytest

from charon_amd import _lib
from charon_amd._lib import BAD_PUBKEY, BAD_SIGNATURE, NOT_VERIFIED, OK

pytestmark = pytest.mark.gpu


def _p(x):
    if x is None:
        return None
    if isinstance(x, np.ndarray):
        return ctypes.c_void_p(x.ctypes.data)
    return ctypes.c_void_p(x.data_ptr())


def _chk(L, rc):
    assert rc == 0, L.hbls_last_error().decode()


def _off_subgroup_g2(rng, count):
    """On-curve G2 points outside the r-torsion, compressed (oracle: test infrastructure)."""
    from oracle import bls12381 as B
    out = []
    while len(out) < count:
        x = (rng.randrange(B.P), rng.randrange(B.P))
        rhs = B.f2_add(B.f2_mul(B.f2_sqr(x), x), B.B_G2)
        y = B.f2_sqrt(rhs)
        if y is None:
            continue
        pt = (x, y)
        if B.g2_in_subgroup(pt):
            continue
        out.append(B.g2_compress(pt))
    return out


@pytest.fixture(scope="module")
def L():
    from charon_amd import tbls
    tbls.HIPBLS()  # initialises the library on its devices
    return _lib.load_library()


def _sign(L, sks, msgs):
    n = len(msgs) // 32
    out = np.zeros(96 * n, dtype=np.uint8)
    st = np.zeros(n, dtype=np.uint8)
    off = np.arange(n, dtype=np.uint64) * 32
    ln = np.full(n, 32, dtype=np.uint32)
    _chk(L, L.hbls_sign_batch(_p(sks), _p(msgs), _p(off), _p(ln), n, _p(out), _p(st)))
    assert not st.any()
    return out


def _pks(L, sks):
    n = len(sks) // 32
    out = np.zeros(48 * n, dtype=np.uint8)
    st = np.zeros(n, dtype=np.uint8)
    _chk(L, L.hbls_secret_to_public_key_batch(_p(sks), n, _p(out), _p(st)))
    assert not st.any()
    return out


@pytest.fixture
def fe_mode(L, request):
    """Batched final exponentiation on (the default at these sizes) or off for the test; slot_msm:
    first the slot-wide check (one multi-scalar multiplication for the signature side, one final
    exponentiation for the call), the per-batch check only when it fails."""
    prev = L.hbls_fe_batch(0 if request.param == "fe_per_group" else 128)
    prev_s = L.hbls_slot_msm(1 if request.param.startswith("slot_msm") else 0)
    # slot_msm_chunks: the combination's public-key side as shared-doubling chunks (k_rlc_msm, a
    # validator's partials per lane) as at C3, instead of one ladder per item
    prev_l = L.hbls_rlc_lanes(4096 if request.param == "slot_msm_chunks" else 0)
    yield request.param
    L.hbls_fe_batch(prev)
    L.hbls_slot_msm(prev_s)
    L.hbls_rlc_lanes(prev_l)


@pytest.mark.parametrize("fe_mode", ["fe_batch", "fe_per_group", "slot_msm", "slot_msm_chunks"], indirect=True)
@pytest.mark.parametrize("key_tables", [False, True], ids=["decompress", "key_tables"])
def test_slot_adversarial_c2(L, key_tables, fe_mode):
    """key_tables: the public keys come from tables made once by hbls_decompress_pubkeys_device
    (the slot's pk_table / dv_pk_table) -- same verdicts and aggregates.  fe_mode: 64 groups per
    final exponentiation, or one per group -- same verdicts."""
    import torch
    from charon_amd import synth
    V, n, t = 10_000, 4, 3
    rng = random.Random(2024)
    cl = synth.make_cluster(V, n, t, n_msgs=64)
    NP = V * n
    M = len(cl.msgs)
    msgs = np.frombuffer(b"".join(cl.msgs), dtype=np.uint8).copy()
    msg_of_v = np.asarray(cl.msg_of_validator, dtype=np.uint32)
    midx = np.repeat(msg_of_v, n)
    item_msgs = msgs.reshape(M, 32)[midx].reshape(-1).copy()
    sks = np.frombuffer(b"".join(cl.share_sks), dtype=np.uint8).copy()
    pks = _pks(L, sks)
    sigs = _sign(L, sks, item_msgs)
    root_sks = np.frombuffer(b"".join(cl.root_sks), dtype=np.uint8).copy()
    root_sigs = _sign(L, root_sks, msgs.reshape(M, 32)[msg_of_v].reshape(-1).copy())
    dv_pks = _pks(L, root_sks)

    # 1 % corrupted partials in equal fifths + 20 undecodable public keys
    bad = rng.sample(range(NP), NP // 100)
    cls = {i: k % 5 for k, i in enumerate(bad)}
    offsub = _off_subgroup_g2(rng, 8)
    expect = np.zeros(NP, dtype=np.uint8)
    wrong_msg = hashlib.sha256(b"some other signing root").digest()
    wm_items = [i for i, c in cls.items() if c == 2]
    wm_sigs = _sign(L, np.concatenate([sks[32 * i:32 * i + 32] for i in wm_items]),
                    np.frombuffer(wrong_msg * len(wm_items), dtype=np.uint8).copy())
    for k, i in enumerate(wm_items):
        sigs[96 * i:96 * i + 96] = wm_sigs[96 * k:96 * k + 96]
    for i, c in cls.items():
        v, s = divmod(i, n)
        if c == 0:
            b = bytearray(rng.randrange(256) for _ in range(96))
            b[0] &= 0x7F  # no compression flag: never decodable
            sigs[96 * i:96 * i + 96] = np.frombuffer(bytes(b), dtype=np.uint8)
            expect[i] = BAD_SIGNATURE
        elif c == 1:
            sigs[96 * i:96 * i + 96] = np.frombuffer(offsub[i % len(offsub)], dtype=np.uint8)
            expect[i] = BAD_SIGNATURE
        elif c == 2:
            expect[i] = NOT_VERIFIED
        elif c == 3:  # a correct partial of another share of the same validator
            j = v * n + (s + 1) % n
            sigs[96 * i:96 * i + 96] = _sign(L, sks[32 * j:32 * j + 32].copy(), msgs.reshape(M, 32)[midx[i]].copy())
            expect[i] = NOT_VERIFIED
        else:
            sigs[96 * i:96 * i + 96] = 0
            sigs[96 * i] = 0xC0
            expect[i] = NOT_VERIFIED
    bad_pk = [i for i in rng.sample(range(NP), 20) if i not in cls]
    for i in bad_pk:
        pks[48 * i] = 0x9A  # compressed, x >= p
        pks[48 * i + 1:48 * i + 48] = 0xFF
        expect[i] = BAD_PUBKEY

    ta_src = (np.arange(V)[:, None] * n + np.arange(t)[None, :]).reshape(-1).astype(np.uint32)
    ta_idx = np.tile(np.arange(1, t + 1, dtype=np.int64), V)
    grp_off = np.arange(V + 1, dtype=np.uint32) * t
    vgrp_off = np.arange(V + 1, dtype=np.uint32) * n
    exp_ta = np.zeros(V, dtype=np.uint8)
    exp_agg = np.zeros(V, dtype=np.uint8)
    for v in range(V):
        mem = [cls.get(v * n + s) for s in range(t)]  # the aggregation sees signatures only
        if any(c in (0, 1) for c in mem):
            exp_ta[v] = BAD_SIGNATURE
            exp_agg[v] = BAD_SIGNATURE
        elif any(c is not None for c in mem):
            exp_agg[v] = NOT_VERIFIED  # decodable but wrong members: a wrong aggregate

    dev = torch.device("cuda", 0)

    def up(a):
        return torch.from_numpy(a).to(dev)

    d = {k: up(a) for k, a in dict(msgs=msgs, moff=(np.arange(M, dtype=np.uint64) * 32).view(np.int64),
                                   mlen=np.full(M, 32, dtype=np.uint32).view(np.int32), pks=pks, sigs=sigs,
                                   midx=midx.view(np.int32), vgoff=vgrp_off.view(np.int32), tsrc=ta_src.view(np.int32),
                                   tidx=ta_idx, goff=grp_off.view(np.int32), dvpk=dv_pks).items()}
    hm = torch.zeros(M * L.hbls_hm_entry_bytes(), dtype=torch.uint8, device=dev)
    vst = torch.full((NP,), 255, dtype=torch.uint8, device=dev)
    tout = torch.zeros(V * 96, dtype=torch.uint8, device=dev)
    tst = torch.full((V,), 255, dtype=torch.uint8, device=dev)
    ast = torch.full((V,), 255, dtype=torch.uint8, device=dev)
    slot = _lib.HblsSlot(msgs=_p(d["msgs"]).value, msg_off=_p(d["moff"]).value, msg_len=_p(d["mlen"]).value,
                         n_msgs=M, hm=_p(hm).value, pks=_p(d["pks"]).value, sigs=_p(d["sigs"]).value,
                         msg_idx=_p(d["midx"]).value, n=NP, vgrp_off=_p(d["vgoff"]).value, n_vgroups=V,
                         vstatus=_p(vst).value, ta_sigs=None, ta_src=_p(d["tsrc"]).value,
                         ta_idx=_p(d["tidx"]).value, grp_off=_p(d["goff"]).value, n_groups=V, n_ta_partials=V * t,
                         ta_out=_p(tout).value, ta_status=_p(tst).value, dv_pks=_p(d["dvpk"]).value,
                         agg_vstatus=_p(ast).value)
    s = torch.cuda.Stream(device=dev)
    if key_tables:
        E = L.hbls_pk_entry_bytes()
        tabs = {"pk": torch.zeros(NP * E, dtype=torch.uint8, device=dev),
                "pkst": torch.full((NP,), 255, dtype=torch.uint8, device=dev),
                "dv": torch.zeros(V * E, dtype=torch.uint8, device=dev),
                "dvst": torch.full((V,), 255, dtype=torch.uint8, device=dev)}
        sp0 = ctypes.c_void_p(s.cuda_stream)
        _chk(L, L.hbls_decompress_pubkeys_device(_p(d["pks"]), NP, _p(tabs["pk"]), _p(tabs["pkst"]), sp0))
        _chk(L, L.hbls_decompress_pubkeys_device(_p(d["dvpk"]), V, _p(tabs["dv"]), _p(tabs["dvst"]), sp0))
        slot.pk_table, slot.pk_table_st = _p(tabs["pk"]).value, _p(tabs["pkst"]).value
        slot.dv_pk_table, slot.dv_pk_table_st = _p(tabs["dv"]).value, _p(tabs["dvst"]).value
    _chk(L, L.hbls_slot_device(ctypes.byref(slot), ctypes.c_void_p(s.cuda_stream)))
    s.synchronize()
    got = vst.cpu().numpy()
    mism = np.nonzero(got != expect)[0]
    assert len(mism) == 0, [(int(i), int(got[i]), int(expect[i]), cls.get(int(i))) for i in mism[:10]]
    assert np.array_equal(tst.cpu().numpy(), exp_ta)
    ga = ast.cpu().numpy()
    bad_a = np.nonzero(ga != exp_agg)[0]
    assert len(bad_a) == 0, [(int(v), int(ga[v]), int(exp_agg[v]), [cls.get(int(v) * n + s) for s in range(n)])
                             for v in bad_a[:10]]
    ok_v = np.nonzero(exp_agg == 0)[0]
    to = tout.cpu().numpy().reshape(V, 96)
    assert np.array_equal(to[ok_v], root_sigs.reshape(V, 96)[ok_v])

    # oracle spot check on a sample of corrupted and clean partials
    from oracle import bls12381 as B
    sample = [bad[k] for k in range(5)] + bad_pk[:1] + [int(rng.randrange(NP))]
    for i in sample:
        st = B.verify(bytes(pks[48 * i:48 * i + 48]), bytes(item_msgs[32 * i:32 * i + 32]),
                      bytes(sigs[96 * i:96 * i + 96]))
        assert st == got[i], (i, st, got[i])


def test_verify_aggregate_512(L):
    """FastAggregateVerify over 512 public keys per message (sync committee)."""
    rng = random.Random(5)
    G, K = 4, 512
    sks = np.frombuffer(b"".join(rng.randrange(1, 2 ** 250).to_bytes(32, "big") for _ in range(G * K)),
                        dtype=np.uint8).copy()
    pks = _pks(L, sks)
    msgs = [hashlib.sha256(b"sync committee root %d" % g).digest() for g in range(G)]
    item_msgs = np.frombuffer(b"".join(msgs[g] for g in range(G) for _ in range(K)), dtype=np.uint8).copy()
    sigs = _sign(L, sks, item_msgs)
    aggs = np.zeros(96 * G, dtype=np.uint8)
    ast = np.zeros(G, dtype=np.uint8)
    goff = np.arange(G + 1, dtype=np.uint32) * K
    _chk(L, L.hbls_aggregate_batch(_p(sigs), _p(goff), G, _p(aggs), _p(ast)))
    assert not ast.any()
    # group 1: a wrong aggregate (group 2's); group 3: one undecodable key
    aggs2 = aggs.copy()
    aggs2[96:192] = aggs[192:288]
    pks2 = pks.copy()
    pks2[48 * (3 * K + 7)] = 0x9A
    pks2[48 * (3 * K + 7) + 1:48 * (3 * K + 8)] = 0xFF
    mb = np.frombuffer(b"".join(msgs), dtype=np.uint8).copy()
    moff = np.arange(G, dtype=np.uint64) * 32
    mlen = np.full(G, 32, dtype=np.uint32)
    st = np.full(G, 255, dtype=np.uint8)
    _chk(L, L.hbls_verify_aggregate_batch(_p(pks2), _p(goff), _p(aggs2), _p(mb), _p(moff), _p(mlen), G, _p(st)))
    assert list(st) == [OK, NOT_VERIFIED, OK, BAD_PUBKEY]


def test_verify_aggregate_bad_offsets(L):
    pks = np.zeros(48 * 4, dtype=np.uint8)
    sigs = np.zeros(96 * 2, dtype=np.uint8)
    mb = np.zeros(64, dtype=np.uint8)
    moff = np.array([0, 32], dtype=np.uint64)
    mlen = np.array([32, 32], dtype=np.uint32)
    st = np.zeros(2, dtype=np.uint8)
    goff = np.array([0, 3, 2], dtype=np.uint32)  # decreasing
    assert L.hbls_verify_aggregate_batch(_p(pks), _p(goff), _p(sigs), _p(mb), _p(moff), _p(mlen), 2, _p(st)) != 0
    assert b"non-decreasing" in L.hbls_last_error()


def test_concurrent_single_item_callers(hipbls):
    """32 threads, each calling verify with one item (valid or wrong message), as charon's stream
    handlers do; every caller gets its own verdict from the coalesced launches."""
    rng = random.Random(9)
    keys = [hipbls.generate_secret_key() for _ in range(64)]
    msgs = [hashlib.sha256(b"duty %d" % (k % 7)).digest() for k in range(64)]
    sigs = hipbls.sign_batch(keys, msgs)
    pks = [hipbls.secret_to_public_key(k) for k in keys]
    cases = []
    for k in range(256):
        j = rng.randrange(64)
        if rng.random() < 0.2:
            cases.append((pks[j], hashlib.sha256(b"wrong").digest(), sigs[j], NOT_VERIFIED))
        else:
            cases.append((pks[j], msgs[j], sigs[j], OK))
    results = [None] * len(cases)

    def worker(w):
        for c in range(w, len(cases), 32):
            pk, m, s, _ = cases[c]
            results[c] = hipbls.verify_batch([pk], [m], [s])[0]

    th = [threading.Thread(target=worker, args=(w,)) for w in range(32)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert results == [c[3] for c in cases]


def test_device_call_and_host_call_do_not_race(L, hipbls):
    """hbls_verify_device on a side stream, then at once a host-buffer verify with other inputs:
    both verdict arrays are right (the library orders its workspaces by events)."""
    import torch
    dev = torch.device("cuda", 0)
    keys = [hipbls.generate_secret_key() for _ in range(96)]
    m = hashlib.sha256(b"race").digest()
    sigs = hipbls.sign_batch(keys, [m] * 96)
    pks = [hipbls.secret_to_public_key(k) for k in keys]
    # device call: 96 partials over one message, every third signature of another key
    dsig = [sigs[(i + 1) % 96] if i % 3 == 0 else sigs[i] for i in range(96)]
    mt = torch.from_numpy(np.frombuffer(m, dtype=np.uint8).copy()).to(dev)
    moff = torch.zeros(1, dtype=torch.int64, device=dev)
    mlen = torch.full((1,), 32, dtype=torch.int32, device=dev)
    hm = torch.zeros(L.hbls_hm_entry_bytes(), dtype=torch.uint8, device=dev)
    dpk = torch.from_numpy(np.frombuffer(b"".join(pks), dtype=np.uint8).copy()).to(dev)
    ds = torch.from_numpy(np.frombuffer(b"".join(dsig), dtype=np.uint8).copy()).to(dev)
    midx = torch.zeros(96, dtype=torch.int32, device=dev)
    goff = torch.tensor([0, 16, 48, 96], dtype=torch.int32, device=dev)
    vst = torch.full((96,), 255, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(device=dev)
    sp = ctypes.c_void_p(s.cuda_stream)
    _chk(L, L.hbls_hash_to_g2_device(_p(mt), _p(moff), _p(mlen), 1, _p(hm), sp))
    _chk(L, L.hbls_verify_device(_p(dpk), _p(ds), _p(midx), _p(hm), 96, _p(goff), 3, _p(vst), sp))
    # immediately: host call with different inputs (all valid, other message)
    m2 = hashlib.sha256(b"race 2").digest()
    sigs2 = hipbls.sign_batch(keys[:40], [m2] * 40)
    assert hipbls.verify_batch(pks[:40], [m2] * 40, sigs2) == [OK] * 40
    s.synchronize()
    assert list(vst.cpu().numpy()) == [NOT_VERIFIED if i % 3 == 0 else OK for i in range(96)]


def test_concurrent_host_batches_overlap_exactly(hipbls):
    """Five threads (more than the library's three host-call contexts, so some wait for one) each
    call VerifyBatch, ThresholdAggregateBatch and VerifyAggregateBatch on their own inputs at once:
    every result equals the same call made alone (hipbls.hip Hc: each call owns a context, the
    device lock covers only the enqueueing)."""
    rng = random.Random(17)
    n_keys = 48
    keys = [hipbls.generate_secret_key() for _ in range(n_keys)]
    pks = [hipbls.secret_to_public_key(k) for k in keys]
    jobs = []
    for t in range(5):
        msgs = [hashlib.sha256(b"host call %d %d" % (t, i % 9)).digest() for i in range(600)]
        ks = [rng.randrange(n_keys) for _ in range(600)]
        sigs = hipbls.sign_batch([keys[k] for k in ks], msgs)
        sigs = [sigs[(i + 1) % 600] if i % 11 == t else sigs[i] for i in range(600)]  # some wrong
        split = hipbls.threshold_split(keys[t], 5, 3)
        m = hashlib.sha256(b"ta %d" % t).digest()
        parts = sorted((i, hipbls.sign(sk, m)) for i, sk in split.items())
        groups = [dict(parts[j:j + 3]) for j in range(3)] * 20
        va_m = [hashlib.sha256(b"va %d %d" % (t, g)).digest() for g in range(40)]
        va_pk = [[pks[(g + j) % n_keys] for j in range(8)] for g in range(40)]
        va_sig = [hipbls.aggregate(hipbls.sign_batch([keys[(g + j) % n_keys] for j in range(8)], [va_m[g]] * 8))
                  for g in range(40)]
        va_sig[t] = va_sig[t + 1]
        jobs.append(([pks[k] for k in ks], msgs, sigs, groups, va_pk, va_sig, va_m))

    def run(j):
        pk, m, sg, groups, va_pk, va_sig, va_m = j
        v = hipbls.verify_batch(pk, m, sg)
        ta = hipbls.threshold_aggregate_batch(groups)
        va = hipbls.verify_aggregate_batch(va_pk, va_sig, va_m)
        return v, ta, va

    alone = [run(j) for j in jobs]
    got = [None] * len(jobs)

    def worker(k):
        got[k] = run(jobs[k])

    th = [threading.Thread(target=worker, args=(k,)) for k in range(len(jobs))]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert got == alone
    assert all(any(st != OK for st in a[0]) for a in alone)  # the wrong signatures were caught
    assert all(a[2][k] != OK for k, a in enumerate(alone))  # and the wrong aggregates


def _stats(L):
    out = (ctypes.c_uint64 * 6)()
    assert L.hbls_stats(out, 6) == 0
    return list(out)


def test_batched_fe_rejects_cancelling_errors(L, hipbls, monkeypatch):
    """300 items over distinct messages (300 groups of one: 5 batches of 64 groups share their
    final exponentiations).  Two signatures carry opposite errors, sig0 + D and sig1 - D: the
    plain sum of the batch is unchanged, so the batch check must weigh every item by its own
    random coefficient (groups of one included) to reject them -- and it does, exactly those two.
    A clean run of the same size needs no per-group check."""
    from oracle import bls12381 as B
    monkeypatch.setenv("HBLS_STATS", "1")
    n = 300
    keys = [hipbls.generate_secret_key() for _ in range(n)]
    msgs = [hashlib.sha256(b"duty %d" % k).digest() for k in range(n)]
    sigs = hipbls.sign_batch(keys, msgs)
    pks = [hipbls.secret_to_public_key(k) for k in keys]
    s0 = _stats(L)
    assert hipbls.verify_batch(pks, msgs, sigs) == [OK] * n
    d = [b - a for a, b in zip(s0, _stats(L))]
    assert d[1] == n and d[2] == 0 and d[3] == 0, d
    D = B.g2_decompress(sigs[7])
    bad = list(sigs)
    bad[0] = B.g2_compress(B.g2_add(B.g2_decompress(sigs[0]), D))
    bad[1] = B.g2_compress(B.g2_add(B.g2_decompress(sigs[1]), B.g2_neg(D)))
    s0 = _stats(L)
    st = hipbls.verify_batch(pks, msgs, bad)
    assert st == [NOT_VERIFIED if i < 2 else OK for i in range(n)]
    d = [b - a for a, b in zip(s0, _stats(L))]
    # the failing batch's groups checked alone; those are the two items' own checks (groups of one):
    # no item is re-checked
    assert d[3] >= 1 and d[2] == 0, d


def test_slot_msm_clean_and_cancelling_errors(L, hipbls, monkeypatch):
    """The slot-wide check (HBLS_SLOT_MSM) on 300 groups of one: a clean call passes it with no
    per-batch or per-item check; two signatures with opposite errors (sig0 + D, sig1 - D) make it
    fail, and the per-batch check then rejects exactly those two (their groups' checks, no re-check alone).  Then the adaptive choice: the
    next calls skip the slot-wide check (same verdicts) until one passes every batch."""
    from oracle import bls12381 as B
    monkeypatch.setenv("HBLS_STATS", "1")
    prev_f, prev_s = L.hbls_fe_batch(128), L.hbls_slot_msm(1)
    try:
        n = 300
        keys = [hipbls.generate_secret_key() for _ in range(n)]
        msgs = [hashlib.sha256(b"slot duty %d" % k).digest() for k in range(n)]
        sigs = hipbls.sign_batch(keys, msgs)
        pks = [hipbls.secret_to_public_key(k) for k in keys]
        s0 = _stats(L)
        assert hipbls.verify_batch(pks, msgs, sigs) == [OK] * n
        d = [b - a for a, b in zip(s0, _stats(L))]
        assert d[1] == n and d[2] == 0 and d[3] == 0 and d[4] == 1 and d[5] == 0, d
        D = B.g2_decompress(sigs[11])
        bad = list(sigs)
        bad[0] = B.g2_compress(B.g2_add(B.g2_decompress(sigs[0]), D))
        bad[1] = B.g2_compress(B.g2_add(B.g2_decompress(sigs[1]), B.g2_neg(D)))
        s0 = _stats(L)
        st = hipbls.verify_batch(pks, msgs, bad)
        assert st == [NOT_VERIFIED if i < 2 else OK for i in range(n)]
        d = [b - a for a, b in zip(s0, _stats(L))]
        assert d[4] == 1 and d[5] == 1 and d[3] >= 1 and d[2] == 0, d
        # adaptive (HBLS_ADAPTIVE, default on): after a failed slot-wide check the next calls skip it
        # and run the per-batch check directly -- same verdicts -- until one passes every batch
        s0 = _stats(L)
        assert hipbls.verify_batch(pks, msgs, bad) == st
        d = [b - a for a, b in zip(s0, _stats(L))]
        assert d[4] == 0 and d[3] >= 1 and d[2] == 0, d
        s0 = _stats(L)
        assert hipbls.verify_batch(pks, msgs, sigs) == [OK] * n  # clean: skipped, every batch passes
        d = [b - a for a, b in zip(s0, _stats(L))]
        assert d[4] == 0 and d[3] == 0 and d[2] == 0, d
        s0 = _stats(L)
        assert hipbls.verify_batch(pks, msgs, sigs) == [OK] * n  # back to the slot-wide check
        d = [b - a for a, b in zip(s0, _stats(L))]
        assert d[4] == 1 and d[5] == 0 and d[2] == 0, d
    finally:
        L.hbls_fe_batch(prev_f)
        L.hbls_slot_msm(prev_s)


def test_batched_groups_pass_without_fallback(L, hipbls, monkeypatch):
    """Clean partials over a few messages: every verification group passes its combined check,
    no item is re-checked alone (the random linear combination is effective, not just correct).
    (hbls_single_max(0): a call this small would otherwise check every item alone.)"""
    monkeypatch.setenv("HBLS_STATS", "1")
    prev_single = L.hbls_single_max(0)
    keys = [hipbls.generate_secret_key() for _ in range(48)]
    msgs = [hashlib.sha256(b"committee %d" % (k % 3)).digest() for k in range(48)]
    sigs = hipbls.sign_batch(keys, msgs)
    pks = [hipbls.secret_to_public_key(k) for k in keys]
    s0 = _stats(L)
    assert hipbls.verify_batch(pks, msgs, sigs) == [OK] * 48
    d = [b - a for a, b in zip(s0, _stats(L))]
    assert d[0] == 48 and d[1] == 3 and d[2] == 0, d  # 3 groups of 16 (HBLS_GROUP_MAX), no fallback
    # one wrong partial: only its group (16 items) is re-checked alone
    bad = list(sigs)
    bad[5] = sigs[6]
    s0 = _stats(L)
    st = hipbls.verify_batch(pks, msgs, bad)
    assert st == [NOT_VERIFIED if i == 5 else OK for i in range(48)]
    d = [b - a for a, b in zip(s0, _stats(L))]
    assert d[2] == 16, d
    # the default for so small a call: every item its own group (its check the item's verdict),
    # no combination, no re-check
    L.hbls_single_max(prev_single)
    s0 = _stats(L)
    st = hipbls.verify_batch(pks, msgs, bad)
    assert st == [NOT_VERIFIED if i == 5 else OK for i in range(48)]
    d = [b - a for a, b in zip(s0, _stats(L))]
    assert d[0] == 48 and d[1] == 48 and d[2] == 0, d


R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def _rand_sks(rng, count):
    """count random secret keys in [1, r) (32 B big-endian), vectorised."""
    raw = np.frombuffer(rng.randbytes(32 * count), dtype=np.uint8).reshape(count, 32).copy()
    raw[:, 0] &= 0x3F  # < 2^254 < r
    raw[:, 31] |= 1    # nonzero
    return raw.reshape(-1)


def _sk_sum(sks):
    return sum(int.from_bytes(bytes(sks[32 * i:32 * i + 32]), "big") for i in range(len(sks) // 32)) % R_ORDER


def test_verify_aggregate_lock_scale(L):
    """cluster/lock.go:185 at scale: one VerifyAggregate group holding 70 000 public shares (the
    segmented key reduction runs 4 passes), beside the edge groups of FastAggregateVerify:
    empty, single key, identity signature, undecodable signature over a group with a bad key
    (signature checked first), a bad key, keys summing to the identity, wrong message.  Host and
    device entry points must agree; small groups are checked against the oracle."""
    import torch
    rng = random.Random(77)
    K = 70_000
    sks = _rand_sks(rng, K + 1025 + 64 + 33 + 1)
    pks = _pks(L, sks)
    lock_hash = hashlib.sha256(b"cluster lock hash").digest()
    other = hashlib.sha256(b"another root").digest()

    def sig_of(lo, hi, msg):
        s = _sk_sum(sks[32 * lo:32 * hi]).to_bytes(32, "big")
        return bytes(_sign(L, np.frombuffer(s, dtype=np.uint8).copy(), np.frombuffer(msg, dtype=np.uint8).copy()))

    o_big, o_1025, o_64, o_33, o_1 = 0, K, K + 1025, K + 1025 + 64, K + 1025 + 64 + 33
    pk = lambda i: bytes(pks[48 * i:48 * i + 48])  # noqa: E731
    bad_pk = bytes([0x9A]) + b"\xff" * 47
    neg = bytearray(pk(o_1))
    neg[0] ^= 0x20  # the negated key (sign flag flipped)
    keys_1025 = [pk(o_1025 + j) for j in range(1025)]
    keys_1025_bad = list(keys_1025)
    keys_1025_bad[1000] = bad_pk
    bad_sig = bytes([0x80]) + b"\xff" * 95  # x >= p
    inf_sig = bytes([0xC0]) + bytes(95)
    groups = [
        ([pk(o_big + j) for j in range(K)], sig_of(o_big, o_big + K, lock_hash), lock_hash, OK),
        ([], sig_of(o_1, o_1 + 1, lock_hash), lock_hash, NOT_VERIFIED),
        ([pk(o_1)], sig_of(o_1, o_1 + 1, lock_hash), lock_hash, OK),
        ([pk(o_33 + j) for j in range(33)], inf_sig, lock_hash, NOT_VERIFIED),
        (keys_1025_bad, bad_sig, lock_hash, BAD_SIGNATURE),
        (keys_1025_bad, sig_of(o_1025, o_1025 + 1025, lock_hash), lock_hash, BAD_PUBKEY),
        ([pk(o_1), bytes(neg)], sig_of(o_1, o_1 + 1, lock_hash), lock_hash, NOT_VERIFIED),
        ([pk(o_64 + j) for j in range(64)], sig_of(o_64, o_64 + 64, other), lock_hash, NOT_VERIFIED),
        (keys_1025, sig_of(o_1025, o_1025 + 1025, lock_hash), lock_hash, OK),
    ]
    G = len(groups)
    goff = np.zeros(G + 1, dtype=np.uint32)
    for g, grp in enumerate(groups):
        goff[g + 1] = goff[g] + len(grp[0])
    allpk = np.frombuffer(b"".join(k for grp in groups for k in grp[0]), dtype=np.uint8).copy()
    allsig = np.frombuffer(b"".join(grp[1] for grp in groups), dtype=np.uint8).copy()
    mb = np.frombuffer(b"".join(grp[2] for grp in groups), dtype=np.uint8).copy()
    moff = np.arange(G, dtype=np.uint64) * 32
    mlen = np.full(G, 32, dtype=np.uint32)
    st = np.full(G, 255, dtype=np.uint8)
    _chk(L, L.hbls_verify_aggregate_batch(_p(allpk), _p(goff), _p(allsig), _p(mb), _p(moff), _p(mlen), G, _p(st)))
    expect = [grp[3] for grp in groups]
    assert list(st) == expect

    # device entry point, same inputs
    dev = torch.device("cuda", 0)
    up = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    hm = torch.zeros(G * L.hbls_hm_entry_bytes(), dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(device=dev)
    sp = ctypes.c_void_p(s.cuda_stream)
    dmb, dmo, dml = up(mb), up(moff.view(np.int64)), up(mlen.view(np.int32))
    dpk, dsig = up(allpk), up(allsig)
    dst = torch.full((G,), 255, dtype=torch.uint8, device=dev)
    _chk(L, L.hbls_hash_to_g2_device(_p(dmb), _p(dmo), _p(dml), G, _p(hm), sp))
    _chk(L, L.hbls_verify_aggregate_device(_p(dpk), _p(goff), G, _p(dsig), _p(hm), _p(dst), sp))
    s.synchronize()
    assert list(dst.cpu().numpy()) == expect

    from oracle import bls12381 as B
    for g in (1, 2, 3, 6):
        assert B.verify_aggregate(groups[g][0], groups[g][1], groups[g][2]) == expect[g], g


def test_pubkey_cache_same_verdicts(hipbls):
    """Verification with the key cache (hbls_pubkey_cache_add) gives the verdicts of the uncached
    path: cached valid keys, cached undecodable / off-curve keys, uncached keys, mixed in one batch."""
    rng = random.Random(31)
    keys = [hipbls.generate_secret_key() for _ in range(40)]
    msgs = [hashlib.sha256(b"cache %d" % (k % 4)).digest() for k in range(40)]
    sigs = hipbls.sign_batch(keys, msgs)
    pks = [hipbls.secret_to_public_key(k) for k in keys]
    bad_x = bytes([0x9A]) + b"\xff" * 47           # x >= p
    bad_flag = bytes([0x1A]) + pks[3][1:]           # compression flag missing
    items = [(pks[i], msgs[i], sigs[i]) for i in range(40)]
    items[5] = (bad_x, msgs[5], sigs[5])
    items[6] = (bad_flag, msgs[6], sigs[6])
    items[7] = (pks[8], msgs[7], sigs[7])            # wrong key
    items[9] = (pks[9], msgs[9], sigs[10])           # wrong signature
    rng.shuffle(items)
    P, M, S = zip(*items)
    hipbls.clear_pubkey_cache()
    plain = hipbls.verify_batch(P, M, S)
    assert hipbls.cache_pubkeys(pks[:25] + [bad_x, bad_flag]) == 27
    cached = hipbls.verify_batch(P, M, S)
    hipbls.clear_pubkey_cache()
    assert cached == plain
    assert sorted(plain).count(0) == 36


@pytest.mark.parametrize("members", [1, 2, 3, 4])
def test_threshold_aggregate_joint_ladders(L, hipbls, members):
    """ThresholdAggregate of 320 validators x 4 partials through the joint ladders (a lane per
    chunk of `members` members; 1 = one ladder per member): the first 192 validators aggregate the
    same share indices (wave-uniform Lagrange digits: the NAF schedule), the rest a random 4-subset
    of 1..10 each (mixed digits in a wave: the general ladder), one group has an undecodable
    partial.  Every aggregate equals the signature under the validator's secret."""
    rng = random.Random(31 + members)
    V, n, t = 320, 10, 4
    msg = hashlib.sha256(b"joint ladders").digest()
    secrets = [hipbls.generate_secret_key() for _ in range(V)]
    roots = hipbls.sign_batch(secrets, [msg] * V)
    groups, want = [], []
    for v in range(V):
        shares = hipbls.threshold_split(secrets[v], n, t)
        ids = [1, 3, 4, 8] if v < 192 else sorted(rng.sample(range(1, n + 1), t))
        sigs = hipbls.sign_batch([shares[i] for i in ids], [msg] * t)
        groups.append(dict(zip(ids, sigs)))
        want.append((OK, roots[v]))
    groups[200][next(iter(groups[200]))] = b"\x00" * 96  # undecodable member
    want[200] = (BAD_SIGNATURE, None)
    prev = L.hbls_ta_joint(members)
    try:
        outs, sts = hipbls.threshold_aggregate_batch(groups)
    finally:
        L.hbls_ta_joint(prev)
    for v in range(V):
        assert sts[v] == want[v][0], v
        if want[v][0] == OK:
            assert outs[v] == want[v][1], v


@pytest.mark.parametrize("members", [0, 2])
def test_threshold_aggregate_uneven_groups(L, hipbls, members):
    """Groups of 2 and 4 members alternating: the member count divides evenly (3 per group on
    average), yet no group has 3 -- the joint and small-scalar paths (which assume exactly t per
    group) must stand down for the per-member ladders, and every aggregate stays right.  members:
    the joint-ladder knob (0 = auto, 2 = forced joint path)."""
    V, n = 128, 10
    msg = hashlib.sha256(b"uneven groups").digest()
    secrets = [hipbls.generate_secret_key() for _ in range(V)]
    roots = hipbls.sign_batch(secrets, [msg] * V)
    groups = []
    for v in range(V):
        t = 2 if v % 2 == 0 else 4
        shares = hipbls.threshold_split(secrets[v], n, t)
        ids = [1, 3] if t == 2 else [2, 5, 7, 9]
        groups.append(dict(zip(ids, hipbls.sign_batch([shares[i] for i in ids], [msg] * t))))
    prev = L.hbls_ta_joint(members)
    try:
        outs, sts = hipbls.threshold_aggregate_batch(groups)
    finally:
        L.hbls_ta_joint(prev)
    assert sts == [OK] * V
    assert outs == roots


def _tune(L, name, value):
    """hbls_tune: set a latency-path layout by name, return the previous value."""
    prev = ctypes.c_size_t()
    assert L.hbls_tune(name.encode(), value, ctypes.byref(prev)) == 0
    return prev.value


def test_tune_names(L):
    """hbls_tune: every documented name round-trips its value; an unknown name is an error that
    names it (include/hipbls.h)."""
    for name in ("HBLS_HASH_PAIR_MAX", "HBLS_HASH_ONE_LANE", "HBLS_HASH_SPLIT", "HBLS_FE18_MAX", "HBLS_TA_PAIR_MAX",
                 "HBLS_DEC_PAIR_MAX"):
        prev = _tune(L, name, 12345)
        assert _tune(L, name, prev) == 12345, name
    assert L.hbls_tune(b"HBLS_NO_SUCH_KNOB", 1, None) == -1
    assert b"HBLS_NO_SUCH_KNOB" in L.hbls_last_error()


def test_hash_paths_agree(L):
    """hash_to_G2 of 65 536 messages through the staged fast kernels (hashsplit.hip, the default),
    then the first 512 of them again through each kernel of hash.hip (HBLS_HASH_SPLIT=0: the
    one-lane kernel for 65 536 messages, the two-lane one for 512; the latter KAT-pinned through
    Sign).  The points must agree."""
    import torch
    dev = torch.device("cuda", 0)
    n, k = 65536, 512
    msgs = np.frombuffer(b"".join(hashlib.sha256(b"m%d" % i).digest() for i in range(n)), dtype=np.uint8).copy()
    E = L.hbls_hm_entry_bytes()
    dm = torch.from_numpy(msgs).to(dev)
    off = torch.from_numpy((np.arange(n, dtype=np.uint64) * 32).view(np.int64)).to(dev)
    ln = torch.full((n,), 32, dtype=torch.int32, device=dev)
    hm_s = torch.zeros(n * E, dtype=torch.uint8, device=dev)
    hm_a = torch.zeros(n * E, dtype=torch.uint8, device=dev)
    hm_b = torch.zeros(k * E, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(device=dev)
    sp = ctypes.c_void_p(s.cuda_stream)
    _chk(L, L.hbls_hash_to_g2_device(_p(dm), _p(off), _p(ln), n, _p(hm_s), sp))
    s.synchronize()
    _tune(L, "HBLS_HASH_SPLIT", 0)
    try:
        _chk(L, L.hbls_hash_to_g2_device(_p(dm), _p(off), _p(ln), n, _p(hm_a), sp))
        _chk(L, L.hbls_hash_to_g2_device(_p(dm), _p(off), _p(ln), k, _p(hm_b), sp))
        s.synchronize()
    finally:
        _tune(L, "HBLS_HASH_SPLIT", 1)
    a = hm_a.cpu().numpy().reshape(n, E)[:, :208]
    b = hm_b.cpu().numpy().reshape(k, E)[:, :208]
    assert np.array_equal(a[:k], b)  # the same operations: the same (lazily reduced) words

    # the staged kernels compute the same points by other operation orders: compare mod p (the
    # stored coordinates are Montgomery forms in [0, 2p))
    from oracle import bls12381 as B

    def canon(rows):
        w = rows[:, :192].reshape(len(rows), 4, 48)
        return [tuple(int.from_bytes(bytes(c), "little") % B.P for c in r) for r in w], rows[:, 192].tolist()

    hs = hm_s.cpu().numpy().reshape(n, E)[:, :208]
    assert canon(hs) == canon(a)

    # the staged kernels for a call below HBLS_HASH_PAIR_MAX: the cofactor ladders on lane pairs
    # (ec28.h F2Half, the default for 512 messages) and on one lane each give the same points
    hm_p = torch.zeros(k * E, dtype=torch.uint8, device=dev)
    hm_1 = torch.zeros(k * E, dtype=torch.uint8, device=dev)
    _chk(L, L.hbls_hash_to_g2_device(_p(dm), _p(off), _p(ln), k, _p(hm_p), sp))
    prev = _tune(L, "HBLS_HASH_PAIR_MAX", 0)
    try:
        _chk(L, L.hbls_hash_to_g2_device(_p(dm), _p(off), _p(ln), k, _p(hm_1), sp))
        s.synchronize()
    finally:
        _tune(L, "HBLS_HASH_PAIR_MAX", prev)
    hp = hm_p.cpu().numpy().reshape(k, E)[:, :208]
    h1 = hm_1.cpu().numpy().reshape(k, E)[:, :208]
    assert np.array_equal(hp, h1)  # the same formulas and values, products split or not
    assert canon(hp) == canon(a[:k])


def test_small_calls_lane_layouts_agree(L, hipbls):
    """A small Verify batch (the latency path: k_lml with its lane-pair chain and eighteen-lane loop,
    the final exponentiation over eighteen lanes) against the same batch with the six-lane final
    exponentiation (HBLS_FE18_MAX=0) and one-lane hashing ladders (HBLS_HASH_PAIR_MAX=0): the
    statuses agree with each other and with construction."""
    rng = random.Random(77)
    keys = [hipbls.generate_secret_key() for _ in range(24)]
    msgs = [hashlib.sha256(b"small %d" % (k % 9)).digest() for k in range(24)]
    sigs = hipbls.sign_batch(keys, msgs)
    pks = [hipbls.secret_to_public_key(k) for k in keys]
    cases = []
    for j in range(48):
        k = rng.randrange(24)
        if j % 5 == 0:
            cases.append((pks[k], hashlib.sha256(b"wrong %d" % j).digest(), sigs[k], NOT_VERIFIED))
        else:
            cases.append((pks[k], msgs[k], sigs[k], OK))
    pk, m, sg, want = zip(*cases)
    got = hipbls.verify_batch(list(pk), list(m), list(sg))
    fe18, hp = _tune(L, "HBLS_FE18_MAX", 0), _tune(L, "HBLS_HASH_PAIR_MAX", 0)
    try:
        got6 = hipbls.verify_batch(list(pk), list(m), list(sg))
        one = hipbls.verify_batch([pk[1]], [m[1]], [sg[1]])
    finally:
        _tune(L, "HBLS_FE18_MAX", fe18)
        _tune(L, "HBLS_HASH_PAIR_MAX", hp)
    assert list(got) == list(want) == list(got6)
    assert list(one) == [want[1]]


def test_slot_c3_full_size(L):
    """BASELINE configs[2] at full size through the benchmarked entry point: 100 000 validators of
    a 10-operator threshold-7 cluster over distinct messages (1 M partials, the slot-wide check,
    the joint aggregation ladders).  Every partial and every aggregate verifies, every aggregate
    is byte-identical to the root-key signature, and the oracle agrees on a sample: three partial
    verdicts and one aggregate recomputed from its seven members."""
    import sys
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from oracle import bls12381 as B
    wl = bench.WORKLOADS["c3"]
    V = wl["validators"]
    d = bench.setup_inputs(L, wl, V, 0)
    n, t, NP, M = d["n"], d["t"], d["NP"], d["M"]
    dev = torch.device("cuda", 0)

    def up(a):
        return torch.from_numpy(a).to(dev)

    g = {k: up(a) for k, a in dict(msgs=d["msgs"], moff=d["moff"].view(np.int64), mlen=d["mlen"].view(np.int32),
                                   pks=d["pks"], sigs=d["sigs"], midx=d["midx"].view(np.int32),
                                   vgoff=d["vgrp_off"].view(np.int32), tsrc=d["ta_src"].view(np.int32),
                                   tidx=d["ta_idx"], goff=d["grp_off"].view(np.int32), dvpk=d["dv_pks"]).items()}
    hm = torch.zeros(M * L.hbls_hm_entry_bytes(), dtype=torch.uint8, device=dev)
    vst = torch.full((NP,), 255, dtype=torch.uint8, device=dev)
    tout = torch.zeros(V * 96, dtype=torch.uint8, device=dev)
    tst = torch.full((V,), 255, dtype=torch.uint8, device=dev)
    ast = torch.full((V,), 255, dtype=torch.uint8, device=dev)
    slot = _lib.HblsSlot(msgs=_p(g["msgs"]).value, msg_off=_p(g["moff"]).value, msg_len=_p(g["mlen"]).value,
                         n_msgs=M, hm=_p(hm).value, pks=_p(g["pks"]).value, sigs=_p(g["sigs"]).value,
                         msg_idx=_p(g["midx"]).value, n=NP, vgrp_off=_p(g["vgoff"]).value, n_vgroups=V,
                         vstatus=_p(vst).value, ta_sigs=None, ta_src=_p(g["tsrc"]).value,
                         ta_idx=_p(g["tidx"]).value, grp_off=_p(g["goff"]).value, n_groups=V, n_ta_partials=V * t,
                         ta_out=_p(tout).value, ta_status=_p(tst).value, dv_pks=_p(g["dvpk"]).value,
                         agg_vstatus=_p(ast).value)
    s = torch.cuda.Stream(device=dev)
    _chk(L, L.hbls_slot_device(ctypes.byref(slot), ctypes.c_void_p(s.cuda_stream)))
    s.synchronize()
    assert int((vst != 0).sum().item()) == 0
    assert int((tst != 0).sum().item()) == 0 and int((ast != 0).sum().item()) == 0
    assert np.array_equal(tout.cpu().numpy(), d["root_sigs"])
    rng = random.Random(3)
    for i in rng.sample(range(NP), 3):
        st = B.verify(bytes(d["pks"][48 * i:48 * i + 48]), bytes(d["item_msgs"][32 * i:32 * i + 32]),
                      bytes(d["sigs"][96 * i:96 * i + 96]))
        assert st == 0, i
    v = rng.randrange(V)
    members = {int(d["ta_idx"][v * t + k]): bytes(d["ta_sigs"][96 * (v * t + k):96 * (v * t + k + 1)])
               for k in range(t)}
    assert B.threshold_aggregate(members)[1] == bytes(tout[96 * v:96 * v + 96].cpu().numpy())
