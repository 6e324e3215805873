"""The decompressed-signature cache (hbls_sig_cache; hipbls.hip sc_put / sc_get, vbatch.hip
k_sc_write / k_sc_index / k_sc_get) on the GPU: ThresholdAggregate of partials an earlier host-buffer Verify batch
decompressed takes them from the cache, and every aggregate and status equals the uncached run --
with valid partials, undecodable and off-subgroup partials (cached with their rejection status),
members never verified (misses, decompressed), duplicate signatures in one Verify batch, and a ring
smaller than the batch (entries overwritten, stale index slots).  Reference flow:
core/parsigex/parsigex.go:93-98 (Verify) -> core/parsigdb/memory.go:197-225 -> core/sigagg/
sigagg.go:105 (ThresholdAggregate of the stored partials)."""
import hashlib
import json
import os
import random

import pytest

from charon_amd import _lib
from charon_amd._lib import BAD_SIGNATURE, OK

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    from charon_amd import tbls
    tbls.HIPBLS()
    return _lib.load_library()


def _cluster(hipbls, rng, V, n, t, tag):
    msgs = [hashlib.sha256(b"%s %d" % (tag, v)).digest() for v in range(V)]
    secrets = [hipbls.generate_secret_key() for _ in range(V)]
    roots = hipbls.sign_batch(secrets, msgs)
    pks, ms, sigs, groups = [], [], [], []
    for v in range(V):
        shares = hipbls.threshold_split(secrets[v], n, t)
        ids = sorted(rng.sample(range(1, n + 1), t)) if v % 3 else list(range(1, t + 1))
        s = hipbls.sign_batch([shares[i] for i in ids], [msgs[v]] * t)
        groups.append(dict(zip(ids, s)))
        for i, sig in zip(ids, s):
            pks.append(hipbls.secret_to_public_key(shares[i]))
            ms.append(msgs[v])
            sigs.append(sig)
    return pks, ms, sigs, groups, roots


@pytest.mark.parametrize("cap", [1 << 21, 64], ids=["ring_large", "ring_wraps"])
def test_aggregate_after_verify_equals_uncached(L, hipbls, cap):
    rng = random.Random(55)
    V, n, t = 96, 7, 5
    pks, ms, sigs, groups, roots = _cluster(hipbls, rng, V, n, t, b"sigcache")
    with open(os.path.join(os.path.dirname(__file__), "golden", "off_subgroup_g2.json")) as f:
        off = [bytes.fromhex(x) for x in json.load(f)["points"][:2]]
    # bad members: random bytes (undecodable), off-subgroup points; one validator's member is
    # never verified (its bytes are only in the aggregation); duplicates of one partial verified twice
    ids0 = list(groups[4])
    groups[4][ids0[0]] = b"\x8f" + bytes(95)
    groups[9][list(groups[9])[1]] = off[0]
    groups[17][list(groups[17])[2]] = off[1]
    never = hipbls.sign_batch([hipbls.generate_secret_key()], [ms[0]])[0]
    groups[30][list(groups[30])[0]] = never
    flat = [(pk, m, s) for pk, m, s in zip(pks, ms, sigs)]
    flat += [(pks[0], ms[0], groups[4][ids0[0]]), (pks[1], ms[1], off[0]), (pks[2], ms[2], off[1])]
    flat += flat[:5]  # the same signatures twice in one Verify batch
    rng.shuffle(flat)
    P, M, S = zip(*flat)
    prev = L.hbls_sig_cache(0)
    try:
        st_plain = hipbls.verify_batch(P, M, S)
        outs_plain, sts_plain = hipbls.threshold_aggregate_batch(groups)
        assert L.hbls_sig_cache(cap) == 0
        st_cached = hipbls.verify_batch(P, M, S)
        outs_cached, sts_cached = hipbls.threshold_aggregate_batch(groups)
        # again: the second aggregation of the same partials (cache hits only, or misses after a wrap)
        outs_again, sts_again = hipbls.threshold_aggregate_batch(groups)
    finally:
        L.hbls_sig_cache(prev)
    assert st_cached == st_plain
    assert sts_cached == sts_plain == sts_again
    assert outs_cached == outs_plain == outs_again
    bad = {4, 9, 17}  # undecodable / off-subgroup members: the aggregation fails
    for v in range(V):
        if v in bad:
            assert sts_plain[v] != OK, v
        elif v == 30:  # a decodable member under another key: an aggregate, not the root signature
            assert sts_plain[v] == OK and outs_plain[v] != roots[v]
        else:
            assert sts_plain[v] == OK and outs_plain[v] == roots[v], v
    assert sts_plain[4] == BAD_SIGNATURE and sts_plain[9] == BAD_SIGNATURE and sts_plain[17] == BAD_SIGNATURE


def test_aggregate_without_prior_verify(L, hipbls):
    """A cache filled by unrelated partials: every member misses and is decompressed."""
    rng = random.Random(56)
    pks, ms, sigs, groups, roots = _cluster(hipbls, rng, 40, 4, 3, b"other")
    _, _, _, groups2, roots2 = _cluster(hipbls, rng, 40, 4, 3, b"fresh")
    hipbls.verify_batch(pks, ms, sigs)
    outs, sts = hipbls.threshold_aggregate_batch(groups2)
    assert sts == [OK] * 40 and outs == roots2


@pytest.mark.parametrize("cap", [1 << 21, 1024], ids=["ring_large", "index_half_full"])
def test_every_verified_member_hits(L, hipbls, monkeypatch, cap):
    """Every member of an aggregation over just-verified partials is found in the cache (HBLS_STATS
    counters 6 and 7: lookups and hits).  With a 1024-entry ring the 480 partials fill the index
    (2048 slots) to a quarter, so many of them hash onto slots another partial of the same put
    took: a put must never evict its own entries (the one-kernel put lost 4.5 % of a 1M put)."""
    import ctypes
    monkeypatch.setenv("HBLS_STATS", "1")
    rng = random.Random(57)
    V, n, t = 96, 7, 5
    pks, ms, sigs, groups, roots = _cluster(hipbls, rng, V, n, t, b"hits")
    prev = L.hbls_sig_cache(cap)
    try:
        st = hipbls.verify_batch(pks, ms, sigs)
        s0 = (ctypes.c_uint64 * 8)()
        assert L.hbls_stats(s0, 8) == 0
        outs, sts = hipbls.threshold_aggregate_batch(groups)
        s1 = (ctypes.c_uint64 * 8)()
        assert L.hbls_stats(s1, 8) == 0
    finally:
        L.hbls_sig_cache(prev)
    assert st == [OK] * (V * t) and sts == [OK] * V and outs == roots
    assert s1[6] - s0[6] == V * t and s1[7] - s0[7] == V * t, (s1[6] - s0[6], s1[7] - s0[7])
