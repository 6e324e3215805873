"""BASELINE configs[3] and configs[4] at their per-GPU shard size through the benchmarked entry
point (hbls_slot_device), -m gpu.

C4: 1M validators of a 7-operator threshold-5 cluster over 8 GPUs = 125 000 validators per GPU,
    64 committee signing roots (one per committee, as attesters of a slot share AttestationData),
    the aggregated share set a non-prefix 5-subset (bench.py ta_share_positions: its Lagrange
    coefficients are not integers).  875 000 partial Verify + 125 000 ThresholdAggregate + 125 000
    aggregate Verify under the DV keys (core/sigagg/sigagg.go:105,117).
C3 adversarial: configs[2]'s geometry (100 000 validators, 10-of-7, distinct messages, the
    non-prefix share set) with the C5 mix below.
C5: the same shard with 1 % of the partials corrupted in equal fifths (bench.py corrupt: random
    bytes, on-curve points outside G2, wrong message, another share's partial, infinity;
    core/parsigex/parsigex_test.go:285-289, core/sigagg/sigagg_test.go:46-67), every status exact
    against the construction, plus sync-committee VerifyAggregate over 1 953 groups of 512 keys
    (999 936 keys) with corrupted groups, through the host-buffer and the device entry points.

The oracle (oracle/bls12381.py, test infrastructure) recomputes a sample: 16 partial verdicts and 4
aggregates at C4, two partials of every corruption class and the post-aggregate verdict of a
validator with a corrupted member at C5.
"""
import ctypes
import hashlib
import os
import random
import sys

import numpy as np
import pytest

from charon_amd import _lib
from charon_amd._lib import BAD_PUBKEY, BAD_SIGNATURE, NOT_VERIFIED, OK

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


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


@pytest.fixture(scope="module")
def c4(L):
    """The C4 shard's inputs (keys and signatures derived on the GPU by bench.setup_inputs)."""
    import bench
    wl = bench.WORKLOADS["c4"]
    return bench.setup_inputs(L, wl, wl["validators"], 0)


def _run_slot(L, d, sigs=None):
    """One hbls_slot_device call on the bench inputs; (vstatus, ta_status, agg_status, aggregates)."""
    import torch
    dev = torch.device("cuda", 0)
    n, t, V, NP, M = d["n"], d["t"], d["V"], d["NP"], d["M"]

    def up(a):
        return torch.from_numpy(a).to(dev)

    g = {k: up(a) for k, a in dict(msgs=d["msgs"], moff=d["moff"].view(np.int64), mlen=d["mlen"].view(np.int32),
                                   pks=d["pks"], sigs=d["sigs"] if sigs is None else sigs, midx=d["midx"].view(np.int32),
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
    return vst.cpu().numpy(), tst.cpu().numpy(), ast.cpu().numpy(), tout.cpu().numpy().reshape(V, 96)


def _oracle_members(d, v):
    t = d["t"]
    sigs = d["sigs"].reshape(d["NP"], 96)
    return {int(d["ta_idx"][v * t + k]): bytes(sigs[int(d["ta_src"][v * t + k])]) for k in range(t)}


def test_slot_c4_shard_clean(L, c4):
    from oracle import bls12381 as B
    d = c4
    V, NP, n = d["V"], d["NP"], d["n"]
    assert (V, n, d["t"], d["M"]) == (125_000, 7, 5, 64)
    assert [int(x) for x in d["ta_idx"][:5]] != [1, 2, 3, 4, 5]  # a non-prefix share set
    vst, tst, ast, tout = _run_slot(L, d)
    assert int((vst != OK).sum()) == 0
    assert int((tst != OK).sum()) == 0 and int((ast != OK).sum()) == 0
    assert np.array_equal(tout, d["root_sigs"].reshape(V, 96))
    rng = random.Random(44)
    for i in rng.sample(range(NP), 16):
        st = B.verify(bytes(d["pks"][48 * i:48 * i + 48]), bytes(d["item_msgs"][32 * i:32 * i + 32]),
                      bytes(d["sigs"][96 * i:96 * i + 96]))
        assert st == vst[i] == OK, i
    for v in rng.sample(range(V), 4):
        st, agg = B.threshold_aggregate(_oracle_members(d, v))
        assert st == OK and agg == bytes(tout[v]), v


def test_slot_c5_shard_adversarial(L, c4):
    import bench
    from oracle import bls12381 as B
    d = dict(c4)
    d["sigs"] = c4["sigs"].copy()
    bench.corrupt(L, d, 0.01, seed=7)
    V, NP, n, t = d["V"], d["NP"], d["n"], d["t"]
    assert d["n_corrupted"] == NP // 100
    vst, tst, ast, tout = _run_slot(L, d, sigs=d["sigs"])
    bad = np.nonzero(vst != d["exp_v"])[0]
    assert len(bad) == 0, [(int(i), int(vst[i]), int(d["exp_v"][i])) for i in bad[:10]]
    assert np.array_equal(tst, d["exp_ta"])
    assert np.array_equal(ast, d["exp_agg"])
    clean = d["exp_agg"] == OK
    assert clean.sum() > 0.9 * V
    assert np.array_equal(tout[clean], d["root_sigs"].reshape(V, 96)[clean])
    # the classes in the mix: statuses BAD_SIGNATURE, NOT_VERIFIED among partials and aggregates
    assert {int(x) for x in np.unique(d["exp_v"])} == {OK, BAD_SIGNATURE, NOT_VERIFIED}
    assert {int(x) for x in np.unique(d["exp_agg"])} == {OK, BAD_SIGNATURE, NOT_VERIFIED}
    # oracle: two partials of each corruption class (bench.corrupt assigns class k % 5 in sample
    # order, seeded) and one clean partial
    rng = random.Random(7)
    bad_items = rng.sample(range(NP), int(NP * 0.01))
    sample = [bad_items[k] for k in (0, 5, 1, 6, 2, 7, 3, 8, 4, 9)] + [next(i for i in range(NP) if d["exp_v"][i] == OK)]
    for i in sample:
        st = B.verify(bytes(d["pks"][48 * i:48 * i + 48]), bytes(d["item_msgs"][32 * i:32 * i + 32]),
                      bytes(d["sigs"][96 * i:96 * i + 96]))
        assert st == vst[i], (i, st, int(vst[i]))
    # a validator whose aggregated members include a decodable corrupted partial: the oracle's
    # aggregate fails the DV-key verification as the GPU's did
    v = next(v for v in range(V) if d["exp_agg"][v] == NOT_VERIFIED)
    st, agg = B.threshold_aggregate(_oracle_members(d, v))
    assert st == OK and agg == bytes(tout[v])
    root = bytes(d["msgs"].reshape(d["M"], 32)[int(d["midx"][v * n])])
    assert B.verify(bytes(d["dv_pks"][48 * v:48 * v + 48]), root, agg) == NOT_VERIFIED == ast[v]


def test_slot_c5_shard_cancelling_errors(L, c4, monkeypatch):
    """The C5 shard (1 % corrupted) plus, in one clean validator, two partials outside its aggregated
    members carrying opposite errors (sig_a + D, sig_b - D): the plain sum of the validator's
    partials is unchanged, so only the random combination's distinct coefficients reject them.  Two
    calls from a clean adaptive history: the first behind a failing slot-wide check (dense
    coefficients), the second under attack (sparse coefficients, ec28.h RLC_DIGITS) -- both
    reject exactly those two, and every other status stays exact."""
    import bench
    from oracle import bls12381 as B
    d = dict(c4)
    d["sigs"] = c4["sigs"].copy()
    bench.corrupt(L, d, 0.01, seed=11)
    V, n, t = d["V"], d["n"], d["t"]
    exp_v = d["exp_v"].copy()
    voff = np.asarray(d["vgrp_off"], dtype=np.int64)
    members = np.asarray(d["ta_src"], dtype=np.int64).reshape(V, t)
    v = next(v for v in range(V) if d["exp_agg"][v] == OK and
             all(exp_v[i] == OK for i in range(voff[v], voff[v + 1])))
    a, b = [i for i in range(voff[v], voff[v + 1]) if i not in set(members[v].tolist())][:2]
    sig = d["sigs"].reshape(-1, 96)
    j = next(j for j in range(voff[v + 1], len(exp_v)) if exp_v[j] == OK)
    D = B.g2_decompress(bytes(sig[j]))  # a valid point: another validator's clean partial
    sig[a] = np.frombuffer(B.g2_compress(B.g2_add(B.g2_decompress(bytes(sig[a])), D)), dtype=np.uint8)
    sig[b] = np.frombuffer(B.g2_compress(B.g2_add(B.g2_decompress(bytes(sig[b])), B.g2_neg(D))), dtype=np.uint8)
    exp_v[a] = exp_v[b] = NOT_VERIFIED
    for i in (a, b):
        assert B.verify(bytes(d["pks"][48 * i:48 * i + 48]), bytes(d["item_msgs"][32 * i:32 * i + 32]),
                        bytes(sig[i])) == NOT_VERIFIED
    monkeypatch.setenv("HBLS_STATS", "1")
    L.hbls_slot_msm(L.hbls_slot_msm(0))  # a clean adaptive history
    for call in range(2):
        s0 = (ctypes.c_uint64 * 6)()
        assert L.hbls_stats(s0, 6) == 0
        vst, tst, ast, tout = _run_slot(L, d, sigs=d["sigs"])
        s1 = (ctypes.c_uint64 * 6)()
        assert L.hbls_stats(s1, 6) == 0
        assert (s1[4] - s0[4] >= 1) if call == 0 else (s1[4] - s0[4] == 0), call  # slot-wide check, then skipped
        bad = np.nonzero(vst != exp_v)[0]
        assert len(bad) == 0, (call, [(int(i), int(vst[i]), int(exp_v[i])) for i in bad[:10]])
        assert np.array_equal(tst, d["exp_ta"]) and np.array_equal(ast, d["exp_agg"]), call
        assert bytes(tout[v]) == bytes(d["root_sigs"].reshape(V, 96)[v])


def test_slot_groups_of_one_partial_with_folded_aggregate(L):
    """Validator groups of ONE partial (a 1-of-1 cluster) with each aggregate's verification folded
    into its group's check: a wrong DV key fails validator 5's group through its aggregate alone.
    The partial must still verify (a failing group of one is its item's verdict only without a
    folded aggregate), the aggregate alone is NOT_VERIFIED, every other status stays OK."""
    import bench
    d = dict(bench.setup_inputs(L, dict(validators=64, n=1, t=1, distinct=False, n_msgs=4), 64, 0))
    V = d["V"]
    dv = d["dv_pks"].copy().reshape(V, 48)
    dv[5] = dv[6]
    d["dv_pks"] = dv.reshape(-1)
    vst, tst, ast, tout = _run_slot(L, d)
    assert int((vst != OK).sum()) == 0, [int(x) for x in np.nonzero(vst != OK)[0]]
    assert int((tst != OK).sum()) == 0
    assert [int(x) for x in np.nonzero(ast != OK)[0]] == [5] and ast[5] == NOT_VERIFIED
    assert np.array_equal(tout, d["root_sigs"].reshape(V, 96))


def test_slot_c3_adversarial(L, monkeypatch):
    """BASELINE configs[2] geometry with the C5 adversarial mix: 100 000 validators of a 10-operator
    threshold-7 cluster over distinct per-validator messages, the non-prefix aggregated share set
    {1, 2, 3, 4, 8, 9, 10}, 1 % of the 1 M partials corrupted in equal fifths (bench.corrupt), the
    aggregated members among them.  This drives the failure paths at 10-item groups: the failing
    slot-wide check, the per-batch check, the per-group and per-item fallbacks, the 10-member chunk
    ladders, and the small-scalar aggregation over groups with a bad member.  The slot runs twice:
    the second call takes the per-batch check directly (adaptive), its random combination in the
    sparse coefficient format (ec28.h RLC_DIGITS).  Every status is exact against the
    construction; the oracle recomputes two partials of every class, 16 clean partials and 8
    aggregates (clean, with an undecodable member, with a decodable wrong member)."""
    import bench
    from oracle import bls12381 as B
    wl = bench.WORKLOADS["c3"]
    d = bench.setup_inputs(L, wl, wl["validators"], 0)
    V, NP, n, t = d["V"], d["NP"], d["n"], d["t"]
    assert (V, n, t, d["M"]) == (100_000, 10, 7, 100_000)
    assert [int(x) for x in d["ta_idx"][:t]] == [1, 2, 3, 4, 8, 9, 10]
    bench.corrupt(L, d, 0.01, seed=303)
    assert d["n_corrupted"] == NP // 100
    members = np.asarray(d["ta_src"], dtype=np.int64).reshape(V, t)
    rng = random.Random(303)
    bad_items = rng.sample(range(NP), int(NP * 0.01))
    assert len(set(bad_items) & set(members.reshape(-1).tolist())) > 0.6 * len(bad_items)  # aggregated members
    monkeypatch.setenv("HBLS_STATS", "1")
    L.hbls_slot_msm(L.hbls_slot_msm(0))  # a clean adaptive history (an earlier test may leave it under attack)
    for call in range(2):
        s0 = (ctypes.c_uint64 * 6)()
        assert L.hbls_stats(s0, 6) == 0
        vst, tst, ast, tout = _run_slot(L, d, sigs=d["sigs"])
        s1 = (ctypes.c_uint64 * 6)()
        assert L.hbls_stats(s1, 6) == 0
        tried, failed = s1[4] - s0[4], s1[5] - s0[5]
        assert (tried >= 1 and failed >= 1) if call == 0 else tried == 0, (call, tried, failed)
        bad = np.nonzero(vst != d["exp_v"])[0]
        assert len(bad) == 0, [(int(i), int(vst[i]), int(d["exp_v"][i])) for i in bad[:10]]
        assert np.array_equal(tst, d["exp_ta"])
        assert np.array_equal(ast, d["exp_agg"])
        clean = d["exp_agg"] == OK
        assert np.array_equal(tout[clean], d["root_sigs"].reshape(V, 96)[clean])
    assert {int(x) for x in np.unique(d["exp_agg"])} == {OK, BAD_SIGNATURE, NOT_VERIFIED}
    # the host-buffer entry points on the same slot: the 1 M-item Verify in chunks over the host-call
    # contexts (hipbls.hip verify_large, deferred Miller lines), then ThresholdAggregate taking its
    # members from the decompressed-signature cache -- every status exact, clean aggregates equal
    hst = np.zeros(NP, dtype=np.uint8)
    assert L.hbls_verify_batch(_p(d["pks"]), _p(d["sigs"]), _p(d["item_msgs"]), _p(d["item_off"]), _p(d["item_len"]),
                               NP, _p(hst)) == 0, L.hbls_last_error()
    bad = np.nonzero(hst != d["exp_v"])[0]
    assert len(bad) == 0, [(int(i), int(hst[i]), int(d["exp_v"][i])) for i in bad[:10]]
    hout = np.zeros(V * 96, dtype=np.uint8)
    hts = np.zeros(V, dtype=np.uint8)
    assert L.hbls_threshold_aggregate_batch(_p(d["ta_sigs"]), _p(d["ta_idx"]), _p(d["grp_off"]), V, _p(hout),
                                            _p(hts)) == 0, L.hbls_last_error()
    assert np.array_equal(hts, d["exp_ta"])
    clean = d["exp_agg"] == OK  # every member valid: the aggregate is the root signature
    assert np.array_equal(hout.reshape(V, 96)[clean], d["root_sigs"].reshape(V, 96)[clean])
    # oracle: two partials of every class (class k % 5 in sample order), 16 clean partials
    sample = [bad_items[k] for k in range(10)]
    cl = random.Random(304)
    sample += cl.sample([i for i in range(NP) if d["exp_v"][i] == OK][:200_000], 16)
    for i in sample:
        st = B.verify(bytes(d["pks"][48 * i:48 * i + 48]), bytes(d["item_msgs"][32 * i:32 * i + 32]),
                      bytes(d["sigs"][96 * i:96 * i + 96]))
        assert st == vst[i] == d["exp_v"][i], (i, st, int(vst[i]))
    # 8 aggregates: 4 clean, 2 with an undecodable member, 2 with a decodable wrong member; each
    # recomputed from its seven members and verified under the DV key by the oracle
    pick = (cl.sample([v for v in range(V) if d["exp_agg"][v] == OK], 4) +
            [v for v in range(V) if d["exp_ta"][v] == BAD_SIGNATURE][:2] +
            [v for v in range(V) if d["exp_agg"][v] == NOT_VERIFIED][:2])
    for v in pick:
        st, agg = B.threshold_aggregate(_oracle_members(d, v))
        assert st == tst[v], v
        if st != OK:
            assert ast[v] == st
            continue
        assert agg == bytes(tout[v]), v
        root = bytes(d["msgs"].reshape(d["M"], 32)[int(d["midx"][v * n])])
        assert B.verify(bytes(d["dv_pks"][48 * v:48 * v + 48]), root, agg) == ast[v], v


def test_host_batches_c5_shard_adversarial(L, c4):
    """The same C5 shard through the host-buffer entry points the Go shim binds
    (hbls_verify_batch over the 875 000 partials, hbls_threshold_aggregate_batch over the 125 000
    groups): every status exact against the construction, aggregates byte-equal to the root-key
    signatures where every member is valid.  Verify runs twice: the first call fails its
    slot-wide check, the second (adaptive) goes straight to the per-batch check -- same statuses."""
    import bench
    d = dict(c4)
    d["sigs"] = c4["sigs"].copy()
    bench.corrupt(L, d, 0.01, seed=11)
    V, NP = d["V"], d["NP"]
    for _ in range(2):
        st = np.full(NP, 255, dtype=np.uint8)
        _chk(L, L.hbls_verify_batch(_p(d["pks"]), _p(d["sigs"]), _p(d["item_msgs"]), _p(d["item_off"]),
                                    _p(d["item_len"]), NP, _p(st)))
        bad = np.nonzero(st != d["exp_v"])[0]
        assert len(bad) == 0, [(int(i), int(st[i]), int(d["exp_v"][i])) for i in bad[:10]]
    tout = np.zeros(V * 96, dtype=np.uint8)
    tst = np.zeros(V, dtype=np.uint8)
    _chk(L, L.hbls_threshold_aggregate_batch(_p(d["ta_sigs"]), _p(d["ta_idx"]), _p(d["grp_off"]), V, _p(tout),
                                             _p(tst)))
    assert np.array_equal(tst, d["exp_ta"])
    clean = d["exp_agg"] == OK
    assert np.array_equal(tout.reshape(V, 96)[clean], d["root_sigs"].reshape(V, 96)[clean])


def _rand_sks(rng, count):
    raw = np.frombuffer(rng.randbytes(32 * count), dtype=np.uint8).reshape(count, 32).copy()
    raw[:, 0] &= 0x3F  # < 2^254 < r
    raw[:, 31] |= 1
    return raw


def test_sync_committee_verify_aggregate_c5(L):
    """1 953 sync-committee messages x 512 public keys (BASELINE configs[4]), FastAggregateVerify per
    message, with corrupted groups: wrong message, infinity signature, another group's signature,
    an undecodable key, a key swapped for another valid key, an on-curve signature outside G2,
    random signature bytes, and an undecodable signature over a group with an undecodable key
    (signature checked first, herumi.go:323-331)."""
    import json
    import torch
    G, K = 1953, 512
    rng = random.Random(1953)
    sks = _rand_sks(rng, G * K)
    pks = np.zeros(48 * G * K, dtype=np.uint8)
    st = np.zeros(G * K, dtype=np.uint8)
    _chk(L, L.hbls_secret_to_public_key_batch(_p(sks.reshape(-1)), G * K, _p(pks), _p(st)))
    assert not st.any()
    ints = [int.from_bytes(sks[i].tobytes(), "big") for i in range(G * K)]
    sums = [sum(ints[g * K:(g + 1) * K]) % R_ORDER for g in range(G)]
    msgs = [hashlib.sha256(b"sync committee root %d" % g).digest() for g in range(G)]
    sign_msgs = list(msgs)
    sign_msgs[3] = hashlib.sha256(b"another root").digest()  # group 3: signed over another message
    skb = np.frombuffer(b"".join(x.to_bytes(32, "big") for x in sums), dtype=np.uint8).copy()
    mb = np.frombuffer(b"".join(sign_msgs), dtype=np.uint8).copy()
    off = np.arange(G, dtype=np.uint64) * 32
    ln = np.full(G, 32, dtype=np.uint32)
    sigs = np.zeros(96 * G, dtype=np.uint8)
    sst = np.zeros(G, dtype=np.uint8)
    _chk(L, L.hbls_sign_batch(_p(skb), _p(mb), _p(off), _p(ln), G, _p(sigs), _p(sst)))
    assert not sst.any()
    sigs = sigs.reshape(G, 96)
    expect = np.full(G, OK, dtype=np.uint8)
    expect[3] = NOT_VERIFIED
    sigs[10] = 0
    sigs[10, 0] = 0xC0  # infinity
    expect[10] = NOT_VERIFIED
    sigs[40] = sigs[41]  # another group's signature
    expect[40] = NOT_VERIFIED
    pks = pks.reshape(G * K, 48)
    pks[20 * K + 77] = 0xFF
    pks[20 * K + 77, 0] = 0x9A  # compressed flag, x >= p
    expect[20] = BAD_PUBKEY
    pks[50 * K + 5] = pks[51 * K + 5]  # a valid key of another group
    expect[50] = NOT_VERIFIED
    with open(os.path.join(ROOT, "tests", "golden", "off_subgroup_g2.json")) as f:
        offsub = bytes.fromhex(json.load(f)["points"][0])
    sigs[60] = np.frombuffer(offsub, dtype=np.uint8)
    expect[60] = BAD_SIGNATURE
    rb = bytearray(rng.randbytes(96))
    rb[0] &= 0x7F
    sigs[70] = np.frombuffer(bytes(rb), dtype=np.uint8)
    expect[70] = BAD_SIGNATURE
    pks[80 * K] = pks[20 * K + 77]
    sigs[80] = sigs[70]
    expect[80] = BAD_SIGNATURE  # the signature is deserialised before the keys
    goff = np.arange(G + 1, dtype=np.uint32) * K
    mb_v = np.frombuffer(b"".join(msgs), dtype=np.uint8).copy()
    pk_flat = pks.reshape(-1).copy()
    sig_flat = sigs.reshape(-1).copy()
    got = np.full(G, 255, dtype=np.uint8)
    _chk(L, L.hbls_verify_aggregate_batch(_p(pk_flat), _p(goff), _p(sig_flat), _p(mb_v), _p(off), _p(ln), G, _p(got)))
    bad = np.nonzero(got != expect)[0]
    assert len(bad) == 0, [(int(g), int(got[g]), int(expect[g])) for g in bad[:10]]
    # the device entry point (inputs resident in HBM, messages hashed on device) agrees
    dev = torch.device("cuda", 0)
    up = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    d_m, d_o, d_l = up(mb_v), up(off.view(np.int64)), up(ln.view(np.int32))
    hm = torch.zeros(G * L.hbls_hm_entry_bytes(), dtype=torch.uint8, device=dev)
    dst = torch.full((G,), 255, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(device=dev)
    sp = ctypes.c_void_p(s.cuda_stream)
    d_pk, d_sig = up(pk_flat), up(sig_flat)
    _chk(L, L.hbls_hash_to_g2_device(_p(d_m), _p(d_o), _p(d_l), G, _p(hm), sp))
    _chk(L, L.hbls_verify_aggregate_device(_p(d_pk), _p(goff), G, _p(d_sig), _p(hm), _p(dst), sp))
    s.synchronize()
    assert np.array_equal(dst.cpu().numpy(), expect)
