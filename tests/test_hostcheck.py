"""The kernels' per-item arithmetic (charon_amd/csrc/*.h), compiled for the CPU by the test-only
harness tests/native/hostcheck.cpp, against the oracle, the reference KATs and the golden
fixtures.  This is how arithmetic is checked without a GPU; the GPU build of the same source is
checked by tests/test_gpu_parity.py."""
import ctypes
import hashlib
import os
import random

import pytest

from oracle import bls12381 as B

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def hc():
    import os
    from charon_amd.build import build_hostcheck
    # HBLS_HOSTCHECK_LIB: another build of the harness (tests/test_sanitizers.py: ASan + UBSan)
    return ctypes.CDLL(os.environ.get("HBLS_HOSTCHECK_LIB") or build_hostcheck(verbose=False))


def _b(n):
    return ctypes.create_string_buffer(n)


def test_fp_mul_random(hc):
    rng = random.Random(1)
    for _ in range(200):
        a, b = rng.randrange(B.P), rng.randrange(B.P)
        o = _b(48)
        hc.hc_fp_mul(a.to_bytes(48, "big"), b.to_bytes(48, "big"), o)
        assert int.from_bytes(o.raw, "big") == a * b % B.P


def test_fp_mul_edges(hc):
    for a in (0, 1, B.P - 1, B.P - 2, (B.P - 1) // 2):
        for b in (0, 1, B.P - 1, 2):
            o = _b(48)
            hc.hc_fp_mul(a.to_bytes(48, "big"), b.to_bytes(48, "big"), o)
            assert int.from_bytes(o.raw, "big") == a * b % B.P


def test_fp2_sqrt(hc):
    rng = random.Random(2)
    for _ in range(30):
        a = (rng.randrange(B.P), rng.randrange(B.P))
        sq = B.f2_sqr(a)
        o = _b(96)
        assert hc.hc_fp2_sqrt(sq[0].to_bytes(48, "big") + sq[1].to_bytes(48, "big"), o) == 0
        x = (int.from_bytes(o.raw[:48], "big"), int.from_bytes(o.raw[48:], "big"))
        assert B.f2_sqr(x) == sq
        # a non-square must be rejected
        if not B.f2_is_square(a):
            assert hc.hc_fp2_sqrt(a[0].to_bytes(48, "big") + a[1].to_bytes(48, "big"), o) == 1


@pytest.mark.parametrize("n", [0, 1, 11, 31, 32, 33, 55, 56, 64, 100, 300])
def test_hash_to_g2_lengths(hc, n):
    msg = hashlib.sha256(b"len%d" % n).digest() * 10
    msg = msg[:n]
    o = _b(96)
    hc.hc_hash_to_g2(msg, n, o)
    assert o.raw == B.g2_compress(B.hash_to_g2(msg))


def test_sign_kats(hc, kats):
    vecs = [kats["registration"]] + kats["deposit"]
    for v in vecs:
        sk, msg = bytes.fromhex(v["sk"]), bytes.fromhex(v["msg"])
        o = _b(96)
        assert hc.hc_sign(sk, msg, len(msg), o) == 0
        assert o.raw.hex() == v["sig"]
        pk = _b(48)
        hc.hc_sk_to_pk(sk, pk)
        assert pk.raw == B.secret_to_public_key(sk)
        assert hc.hc_verify(pk.raw, msg, len(msg), bytes.fromhex(v["sig"])) == 0


def test_verify_fixtures(hc, fixtures):
    for c in fixtures["verify"]:
        msg = bytes.fromhex(c["msg"])
        st = hc.hc_verify(bytes.fromhex(c["pk"]), msg, len(msg), bytes.fromhex(c["sig"]))
        assert st == c["status"], c["name"]


def test_lock_registration_kats(hc, kats):
    L = kats["locks"][3]
    for v in L["validators"]:
        r = v["registration"]
        msg = bytes.fromhex(r["msg"])
        assert hc.hc_verify(bytes.fromhex(v["dpk"]), msg, len(msg), bytes.fromhex(r["sig"])) == 0


def test_threshold_aggregate_fixtures(hc, fixtures):
    for c in fixtures["threshold_aggregate"]:
        items = list(c["partials"].items())
        if not items or c["name"] == "k1":
            continue  # empty / k=1 semantics live in the kernel driver, not the arithmetic
        sigs = b"".join(bytes.fromhex(v) for _, v in items)
        idx = (ctypes.c_int64 * len(items))(*[int(k) for k, _ in items])
        o = _b(96)
        st = hc.hc_lagrange_g2(sigs, idx, len(items), o)
        assert st == c["status"], c["name"]
        if st == 0:
            assert o.raw.hex() == c["out"], c["name"]


def test_pairing_matches_oracle(hc):
    rng = random.Random(3)
    a, b = rng.randrange(1, B.R), rng.randrange(1, B.R)
    P, Q = B.g1_mul(B.G1_GEN, a), B.g2_mul(B.G2_GEN, b)
    o = _b(576)
    assert hc.hc_pairing(B.g1_compress(P), B.g2_compress(Q), o) == 0
    ours = [int.from_bytes(o.raw[48 * i:48 * i + 48], "big") for i in range(12)]
    e = B.pairing(P, Q)
    e3 = B._p12_mul(B._p12_mul(e, e), e)
    vals = []
    for k in (0, 2, 4, 1, 3, 5):  # tower coefficient of w^k: a + b u with u = w^6 - 1
        bb = e3[k + 6]
        vals += [(e3[k] + bb) % B.P, bb]
    assert vals == ours


def test_rlc_endomorphism_ladders(hc, kats):
    """rlc.h: [a] P + [b] phi(P) == [a + b lambda] P on G1 and [a] S + [b] (-psi^2 S) ==
    [a + b lambda] S on G2 with lambda = -x^2 mod r (the batched verification's coefficients)."""
    lam = (-B.X_PARAM ** 2) % B.R
    rng = random.Random(11)
    for v in kats["deposit"]:
        pk, sig = bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"])
        P, S = B.g1_decompress(pk), B.g2_decompress(sig)
        for a, b in ((rng.getrandbits(32), rng.getrandbits(32)), (0xFFFFFFFF, 0xFFFFFFFF), (1, 0), (0, 1)):
            o48, o96 = _b(48), _b(96)
            assert hc.hc_rlc(pk, sig, a, b, o48, o96) == 0
            r = (a + b * lam) % B.R
            assert o48.raw == B.g1_compress(B.g1_mul(P, r))
            assert o96.raw == B.g2_compress(B.g2_mul(S, r))
