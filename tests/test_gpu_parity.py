"""GPU parity: libhipbls.so (through the C ABI, via charon_amd.tbls) against the reference KATs
and the oracle-generated golden fixtures.  Bit-exact verdicts, byte-exact signatures."""
import hashlib
import io
import random

import pytest

from charon_amd._lib import BAD_SIGNATURE, COMBINE_FAILED, NOT_VERIFIED, OK

pytestmark = pytest.mark.gpu


def test_sign_kats(hipbls, kats):
    vecs = [kats["registration"]] + kats["deposit"]
    sks = [bytes.fromhex(v["sk"]) for v in vecs]
    msgs = [bytes.fromhex(v["msg"]) for v in vecs]
    sigs = hipbls.sign_batch(sks, msgs)
    assert [s.hex() for s in sigs] == [v["sig"] for v in vecs]
    for v in kats["deposit"]:
        assert hipbls.secret_to_public_key(bytes.fromhex(v["sk"])).hex() == v["pk"]


def test_verify_kats(hipbls, kats):
    vecs = [kats["registration"]] + kats["deposit"]
    pks = [hipbls.secret_to_public_key(bytes.fromhex(v["sk"])) for v in vecs]
    st = hipbls.verify_batch(pks, [bytes.fromhex(v["msg"]) for v in vecs], [bytes.fromhex(v["sig"]) for v in vecs])
    assert st == [OK] * len(vecs)


def test_lock_kats(hipbls, kats):
    for L in kats["locks"]:
        pks = [bytes.fromhex(s) for v in L["validators"] for s in v["shares"]]
        hipbls.verify_aggregate(pks, bytes.fromhex(L["signature_aggregate"]), bytes.fromhex(L["lock_hash"]))
        regs = [v for v in L["validators"] if "registration" in v]
        if regs:
            st = hipbls.verify_batch([bytes.fromhex(v["dpk"]) for v in regs],
                                     [bytes.fromhex(v["registration"]["msg"]) for v in regs],
                                     [bytes.fromhex(v["registration"]["sig"]) for v in regs])
            assert st == [OK] * len(regs)


def test_verify_fixtures(hipbls, fixtures):
    cs = fixtures["verify"]
    st = hipbls.verify_batch([bytes.fromhex(c["pk"]) for c in cs], [bytes.fromhex(c["msg"]) for c in cs],
                             [bytes.fromhex(c["sig"]) for c in cs])
    assert {c["name"]: s for c, s in zip(cs, st)} == {c["name"]: c["status"] for c in cs}


def test_threshold_aggregate_fixtures(hipbls, fixtures):
    cs = fixtures["threshold_aggregate"]
    groups = [{int(k): bytes.fromhex(v) for k, v in c["partials"].items()} for c in cs]
    outs, sts = hipbls.threshold_aggregate_batch(groups)
    for c, o, s in zip(cs, outs, sts):
        assert s == c["status"], c["name"]
        if s == OK:
            assert o.hex() == c["out"], c["name"]


def test_aggregate_fixtures(hipbls, fixtures):
    cs = fixtures["aggregate"]
    outs, sts = hipbls.aggregate_batch([[bytes.fromhex(s) for s in c["sigs"]] for c in cs])
    for c, o, s in zip(cs, outs, sts):
        assert s == c["status"], c["name"]
        if s == OK:
            assert o.hex() == c["out"], c["name"]


def test_verify_aggregate_fixtures(hipbls, fixtures):
    cs = fixtures["verify_aggregate"]
    sts = hipbls.verify_aggregate_batch([[bytes.fromhex(p) for p in c["pks"]] for c in cs],
                                        [bytes.fromhex(c["sig"]) for c in cs], [bytes.fromhex(c["msg"]) for c in cs])
    assert {c["name"]: s for c, s in zip(cs, sts)} == {c["name"]: c["status"] for c in cs}


def test_tbls_suite_threshold_aggregate(hipbls):
    """tbls_test.go:72-97: split 5/3, sign each share, ThresholdAggregate == Sign(secret)."""
    data = b"hello obol!"
    secret = hipbls.generate_secret_key()
    total = hipbls.sign(secret, data)
    shares = hipbls.threshold_split(secret, 5, 3)
    sigs = {i: hipbls.sign(k, data) for i, k in shares.items()}
    assert hipbls.threshold_aggregate(sigs) == total
    assert hipbls.recover_secret(shares, 5, 3) == secret
    hipbls.verify(hipbls.secret_to_public_key(secret), data, total)


def test_tbls_suite_verify_aggregate(hipbls):
    """tbls_test.go:129-167."""
    data = b"hello obol!"
    keys = [hipbls.generate_secret_key() for _ in range(10)]
    sigs = [hipbls.sign(k, data) for k in keys]
    hipbls.verify_aggregate([hipbls.secret_to_public_key(k) for k in keys], hipbls.aggregate(sigs), data)


def test_threshold_split_insecure_deterministic(hipbls):
    seed = hashlib.sha256(b"insecure").digest() * 8
    s1 = hipbls.threshold_split_insecure(seed[:32], 4, 3, io.BytesIO(seed[32:]))
    s2 = hipbls.threshold_split_insecure(seed[:32], 4, 3, io.BytesIO(seed[32:]))
    assert s1 == s2 and len(s1) == 4


def test_error_strings(hipbls, fixtures):
    from charon_amd.tbls import TblsError
    c = {x["name"]: x for x in fixtures["verify"]}
    with pytest.raises(TblsError, match="signature not verified"):
        x = c["wrong_message"]
        hipbls.verify(bytes.fromhex(x["pk"]), bytes.fromhex(x["msg"]), bytes.fromhex(x["sig"]))
    with pytest.raises(TblsError, match="cannot unmarshal signature into Herumi signature"):
        x = c["off_subgroup_sig"]
        hipbls.verify(bytes.fromhex(x["pk"]), bytes.fromhex(x["msg"]), bytes.fromhex(x["sig"]))
    with pytest.raises(TblsError, match="cannot set compressed public key in Herumi format"):
        x = c["pk_off_subgroup"]
        hipbls.verify(bytes.fromhex(x["pk"]), bytes.fromhex(x["msg"]), bytes.fromhex(x["sig"]))
    with pytest.raises(TblsError, match="cannot combine signatures"):
        hipbls.threshold_aggregate({})


def test_batch_mixed_random(hipbls):
    """A few hundred partials with a deterministic mix of corruptions; verdicts must match the
    expected class exactly (valid -> OK, wrong msg / wrong index -> NOT_VERIFIED, garbage ->
    BAD_SIGNATURE)."""
    rng = random.Random(7)
    n_val, n, t = 32, 4, 3
    secrets_ = [hipbls.generate_secret_key() for _ in range(n_val)]
    msgs = [hashlib.sha256(b"m%d" % (v % 5)).digest() for v in range(n_val)]
    pks, ms, sigs, expect = [], [], [], []
    share_sets = [hipbls.threshold_split(s, n, t) for s in secrets_]
    all_sks = [share_sets[v][i] for v in range(n_val) for i in range(1, n + 1)]
    all_msgs = [msgs[v] for v in range(n_val) for _ in range(n)]
    all_sigs = hipbls.sign_batch(all_sks, all_msgs)
    all_pks = [hipbls.secret_to_public_key(k) for k in all_sks]
    for j, (pk, m, s) in enumerate(zip(all_pks, all_msgs, all_sigs)):
        r = rng.random()
        if r < 0.1:
            s = bytes(rng.randrange(256) for _ in range(96))
            s = bytes([s[0] & 0x7F]) + s[1:]  # clear compression flag: always undecodable
            exp = BAD_SIGNATURE
        elif r < 0.2:
            m = hashlib.sha256(b"wrong").digest()
            exp = NOT_VERIFIED
        elif r < 0.3:
            pk = all_pks[j ^ 1]
            exp = NOT_VERIFIED
        else:
            exp = OK
        pks.append(pk)
        ms.append(m)
        sigs.append(s)
        expect.append(exp)
    assert hipbls.verify_batch(pks, ms, sigs) == expect
    # threshold aggregate every validator from its first t partials, then verify under the DV key
    groups = [{i: all_sigs[v * n + i - 1] for i in range(1, t + 1)} for v in range(n_val)]
    outs, sts = hipbls.threshold_aggregate_batch(groups)
    assert sts == [OK] * n_val
    assert outs == hipbls.sign_batch(secrets_, msgs)
    assert hipbls.verify_batch([hipbls.secret_to_public_key(s) for s in secrets_], msgs, outs) == [OK] * n_val


def test_lane_pair_subgroup_checks(hipbls, fixtures, kats):
    """The subgroup checks with each item's ladder split over a lane pair (hbls_dec_pair_max; the
    non-default small-call path of vbatch.hip k_g1_subgroup_h / k_g2_subgroup_h) give the same
    verdicts: the fixtures (off-subgroup keys and signatures, every encoding reject), the KATs, and
    the off-subgroup G2 points, in batches below and above a pair threshold of 8."""
    import json
    import os

    from charon_amd import _lib
    L = _lib.load_library()
    cs = fixtures["verify"]
    P = [bytes.fromhex(c["pk"]) for c in cs]
    M = [bytes.fromhex(c["msg"]) for c in cs]
    S = [bytes.fromhex(c["sig"]) for c in cs]
    exp = [c["status"] for c in cs]
    with open(os.path.join(os.path.dirname(__file__), "golden", "off_subgroup_g2.json")) as f:
        off = [bytes.fromhex(x) for x in json.load(f)["points"]]
    vecs = [kats["registration"]] + kats["deposit"]
    kp = [hipbls.secret_to_public_key(bytes.fromhex(v["sk"])) for v in vecs]
    km = [bytes.fromhex(v["msg"]) for v in vecs]
    ks = [bytes.fromhex(v["sig"]) for v in vecs]
    P2, M2, S2 = kp + kp[:1] * len(off), km + km[:1] * len(off), ks + off
    exp2 = [OK] * len(vecs) + [BAD_SIGNATURE] * len(off)
    prev = L.hbls_dec_pair_max(1 << 30)
    try:
        assert hipbls.verify_batch(P, M, S) == exp
        assert hipbls.verify_batch(P2, M2, S2) == exp2
        L.hbls_dec_pair_max(8)  # a batch above it keeps the one-lane kernels, one below takes pairs
        assert hipbls.verify_batch(P[:6], M[:6], S[:6]) == exp[:6]
        assert hipbls.verify_batch(P, M, S) == exp
    finally:
        L.hbls_dec_pair_max(prev)
    assert hipbls.verify_batch(P, M, S) == exp


def test_c_client(kats):
    """A C program through include/hipbls.h (tests/native/cabi_client.c, built by
    charon_amd/build.py with -std=c99 -Werror; what the Go shim's cgo does, without Python): it
    signs the reference's teku registration root with the teku key (byte-equal to the teku
    signature), verifies it and a corrupted copy (the status the oracle gives), finds the first
    failure of that pair, and threshold-aggregates a 3-of-4 split over shares {2, 3, 4} back to the
    key's own signature."""
    import json
    import subprocess
    from charon_amd.build import build_c_client
    from oracle import bls12381 as B
    r = kats["registration"]
    exe = build_c_client(verbose=False)
    p = subprocess.run([exe, r["sk"], r["msg"], r["sig"]], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    out = json.loads(p.stdout.strip().splitlines()[-1])
    bad = bytearray(bytes.fromhex(r["sig"]))
    bad[95] ^= 1
    pk = B.secret_to_public_key(bytes.fromhex(r["sk"]))
    want_bad = B.verify(pk, bytes.fromhex(r["msg"]), bytes(bad))
    assert out["sign_equals_teku"] is True
    assert out["verify"] == [0, want_bad] and want_bad != 0
    assert out["first_error"] == [1, out["verify"][1]]
    assert out["aggregate_status"] == 0 and out["aggregate_equals_signature"] is True
    assert out["build"].startswith("hbls-build:")
