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


def test_fp2_mul_lazy_bounds(hc):
    """The Fp2 product and square on lazily reduced operands (any value below 2p, the kernels'
    invariant), extremes included: result = a b / 2^392 mod p and below 2p."""
    P, R_INV = B.P, pow(2, -392, B.P)
    top = 2 * P - 1
    vals = [0, 1, 2, P - 1, P, P + 1, top, top - 1, (1 << 381) - 1, (1 << 380), 2 * P - (1 << 200)]
    rng = random.Random(7)
    pairs = [((x, y), (u, v)) for x in vals[::2] for y in vals[1::2] for u in (top, 0, P) for v in (top, 1, P - 1)]
    pairs += [((rng.randrange(2 * P), rng.randrange(2 * P)), (rng.randrange(2 * P), rng.randrange(2 * P)))
              for _ in range(300)]
    for (a0, a1), (b0, b1) in pairs:
        o, q = _b(96), _b(96)
        hc.hc_fp2_mul_raw(a0.to_bytes(48, "big") + a1.to_bytes(48, "big"),
                          b0.to_bytes(48, "big") + b1.to_bytes(48, "big"), o, q)
        r = (int.from_bytes(o.raw[:48], "big"), int.from_bytes(o.raw[48:], "big"))
        s = (int.from_bytes(q.raw[:48], "big"), int.from_bytes(q.raw[48:], "big"))
        assert r[0] % P == (a0 * b0 - a1 * b1) * R_INV % P and r[1] % P == (a0 * b1 + a1 * b0) * R_INV % P
        assert s[0] % P == (a0 * a0 - a1 * a1) * R_INV % P and s[1] % P == 2 * a0 * a1 * R_INV % P
        assert max(r + s) < 2 * P


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


def _lagrange(ids):
    lam = []
    for j in ids:
        num, den = 1, 1
        for m in ids:
            if m != j:
                num, den = num * m % B.R, den * (m - j) % B.R
        lam.append(num * pow(den, -1, B.R) % B.R)
    return lam


def test_ta_small_split(hc):
    """ta_small.h: lambda_j(0) = s c_j (mod r) with small integers c_j for every index set a
    cluster of up to 10 operators can aggregate (and random larger ones); refused for index 0,
    duplicates and sizes outside 2..16 (the general path runs there)."""
    import itertools
    rng = random.Random(8)
    sets = [list(c) for t in range(2, 11) for c in itertools.combinations(range(1, 11), t)]
    sets = rng.sample(sets, 300) + [[1, 2, 3, 4, 8, 9, 10], [1, 3, 4, 8], [-3, 5, 7], [1, 64, 2 ** 20]]
    sets += [rng.sample(range(1, 65), rng.randrange(2, 17)) for _ in range(40)]
    c = (ctypes.c_int64 * 16)()
    s = _b(32)
    worst = 0
    for ids in sets:
        arr = (ctypes.c_int64 * len(ids))(*ids)
        if not hc.hc_ta_small(arr, len(ids), c, s):
            assert max(map(abs, ids)) > 10, ids  # only large index sets may overflow 63 bits
            continue
        sv = int.from_bytes(s.raw, "big")
        for j, lam in enumerate(_lagrange(ids)):
            assert lam == sv * c[j] % B.R, (ids, j)
        if max(map(abs, ids)) <= 10:
            worst = max(worst, max(abs(c[j]) for j in range(len(ids))))
    assert 0 < worst < 2 ** 22
    # E_j = -2^63 exactly for x_j = -2^30 (no multiplication overflows, but |E_j| does not fit)
    edge = [-2 ** 30, 2 ** 30, -2 ** 30 + 1, -2 ** 30 + 4]
    e0 = edge[0]
    for m in edge[1:]:
        e0 *= m - edge[0]
    assert e0 == -2 ** 63
    for bad in ([0, 1, 2], [1, 1, 2], [5], list(range(1, 18)), edge):
        arr = (ctypes.c_int64 * len(bad))(*bad)
        assert hc.hc_ta_small(arr, len(bad), c, s) == 0, bad


def test_ta_small_aggregate_matches_lagrange(hc, fixtures):
    """[s](sum_j [c_j] sigma_j) == sum_j [lambda_j] sigma_j, byte for byte, on the golden
    ThresholdAggregate fixtures and a 7-of-10 non-prefix set."""
    checked = 0
    for case in fixtures["threshold_aggregate"]:
        items = list(case["partials"].items())
        if case["status"] != 0 or len(items) < 2:
            continue
        sigs = b"".join(bytes.fromhex(v) for _, v in items)
        idx = (ctypes.c_int64 * len(items))(*[int(k) for k, _ in items])
        o = _b(96)
        st = hc.hc_lagrange_g2_small(sigs, idx, len(items), o)
        if st == 7:
            continue
        assert st == 0 and o.raw.hex() == case["out"], case["name"]
        checked += 1
    assert checked >= 1
    secret = 0x1234567890ABCDEF % B.R
    coeffs = [0x1111 * k + 7 for k in range(1, 7)]
    msg = hashlib.sha256(b"ta small").digest()
    ids = [1, 2, 3, 4, 8, 9, 10]
    shares = {i: (secret + sum(a * i ** (k + 1) for k, a in enumerate(coeffs))) % B.R for i in ids}
    sigs = b"".join(B.sign(shares[i].to_bytes(32, "big"), msg) for i in ids)
    idx = (ctypes.c_int64 * 7)(*ids)
    o = _b(96)
    assert hc.hc_lagrange_g2_small(sigs, idx, 7, o) == 0
    assert o.raw == B.sign(secret.to_bytes(32, "big"), msg)


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


def test_fp_inv_divsteps(hc):
    """fp.h fp_inv (Bernstein-Yang divsteps, 30 per batch, stopping once g = 0) equals a^(p-2) and the
    oracle's inverse on 0, 1, p - 1, small values, powers of two, values near 2^380 and 2000 random
    values, within the FP_INV_BATCHES bound (with room to spare); the fixed-trip version of the
    secret-key paths (fp_inv_ct) gives the same inverse after always FP_INV_BATCHES batches"""
    hc.hc_fp_inv.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int),
                             ctypes.POINTER(ctypes.c_int)]
    rng = random.Random(30)
    vals = [0, 1, 2, 3, B.P - 1, B.P - 2, (B.P + 1) // 2] + [1 << k for k in range(0, 381, 17)]
    vals += [(1 << 380) + d for d in (-1, 0, 1)] + [rng.randrange(B.P) for _ in range(2000)]
    worst = 0
    for x in vals:
        out = ctypes.create_string_buffer(144)
        nb, nct = ctypes.c_int(0), ctypes.c_int(0)
        hc.hc_fp_inv(x.to_bytes(48, "big"), out, ctypes.byref(nb), ctypes.byref(nct))
        want = pow(x, B.P - 2, B.P)
        assert int.from_bytes(out.raw[:48], "big") == want, x
        assert int.from_bytes(out.raw[48:96], "big") == want, x
        assert int.from_bytes(out.raw[96:], "big") == want, x
        assert nct.value == 40, nct.value
        worst = max(worst, nb.value)
    assert worst <= 34, worst  # FP_INV_BATCHES = 40


def test_host_mul64_matches_r28(hc):
    """hostmul64.h (the host builds' 64-bit Montgomery products: the CPU baseline and this harness)
    returns bit for bit what the 28-bit cores of fp.h / ec28.h return: stored-word products and
    squares, the Fp2 product with its signed real part, 28-bit-limb products on normalised and
    lazy limbs, the lazy Fp2 dot product, f2l_mul and the paired products / squares of the G1
    formulas (ec28.h mul28x2_core)"""
    hc.hc_mul64_selftest.argtypes = [ctypes.c_int, ctypes.c_uint64]
    assert hc.hc_mul64_selftest(4000, 2834) == 0

