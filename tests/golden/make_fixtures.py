"""Generate tests/golden/fixtures_small.json with the Python oracle (oracle/bls12381.py).

Cases (status codes as in include/hipbls.h):
  verify:  valid / wrong message / wrong share index / random 96 bytes / all-zero signature /
           off-subgroup G2 signature / infinity signature / infinity public key /
           x >= p / no-sqrt x / missing compression flag / off-subgroup G1 pk /
           non-canonical infinity / 11-byte "hello obol!" message (tbls_test.go:73) /
           the G2-side encoding rejects: x.c1 >= p, x.c0 >= p, no square root, compression
           flag clear, infinity with nonzero bits (three placements), a flipped sign bit
  threshold_aggregate: t-of-n subsets, n > t (sigagg_test.go passes all n), k = 1, index 0,
           negative index, undecodable partial, empty group, a member of every G2-side
           encoding class
  aggregate / verify_aggregate: tbls_test.go:129-167 shape (10 keys), empty inputs
Deterministic (seeded); run time ~2-3 minutes.

Parity status: the valid / wrong-message / wrong-key / random-bytes cases follow from the
ciphersuite the reference KATs pin (tests/golden/kat_reference.json).  The edge cases no reference
test pins -- off-subgroup points, infinity encodings, non-canonical flags, share index 0 or
negative, k = 0 / 1, empty Aggregate / VerifyAggregate -- are "parity unpinned": they follow the
decision rules of SURVEY.md Appendix A (herumi's believed ETH-mode behaviour), since herumi
(bls-eth-go-binary v1.36.1) is absent offline.
"""

from __future__ import annotations

import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))

from oracle import bls12381 as B  # noqa: E402

rng = random.Random(0x5EEDC4A7)


def rand_sk() -> bytes:
    return rng.randrange(1, B.R).to_bytes(32, "big")


def off_subgroup_g2() -> bytes:
    while True:
        x = (rng.randrange(B.P), rng.randrange(B.P))
        y = B.f2_sqrt(B.f2_add(B.f2_mul(B.f2_sqr(x), x), B.B_G2))
        if y is not None:
            pt = (x, y)
            if not B.g2_in_subgroup(pt):
                return B.g2_compress(pt)


def off_subgroup_g1() -> bytes:
    while True:
        x = rng.randrange(B.P)
        y = B.fp_sqrt(x * x * x + 4)
        if y is not None and not B.g1_in_subgroup((x, y)):
            return B.g1_compress((x, y))


def no_sqrt_x_g1() -> bytes:
    while True:
        x = rng.randrange(B.P)
        if B.fp_sqrt(x * x * x + 4) is None:
            b = bytearray(x.to_bytes(48, "big"))
            b[0] |= 0x80
            return bytes(b)


def g2_bytes(x0: int, x1: int, flags: int = 0x80) -> bytearray:
    """ZCash G2 layout: x.c1 then x.c0, 48 B each, flags in the top three bits."""
    b = bytearray(x1.to_bytes(48, "big") + x0.to_bytes(48, "big"))
    b[0] |= flags
    return b


def no_sqrt_x_g2(r: random.Random) -> bytes:
    while True:
        x = (r.randrange(B.P), r.randrange(B.P))
        if B.f2_sqrt(B.f2_add(B.f2_mul(B.f2_sqr(x), x), B.B_G2)) is None:
            return bytes(g2_bytes(*x))


def g2_encoding_rejects(sig: bytes, r: random.Random):
    """The Sign.Deserialize rejects behind herumi.go:294-297 (parsigex_test.go:285-289 feeds
    undecodable partials): (name, 96 bytes) -- x.c1 >= p, x.c0 >= p, no square root, compression
    flag clear, infinity with nonzero bits, plus a flipped sign bit (a valid point, -sigma)."""
    x1 = int.from_bytes(sig[:48], "big") & ((1 << 381) - 1)
    x0 = int.from_bytes(sig[48:], "big")
    out = [("sig_x_c1_ge_p", bytes(g2_bytes(x0, x1 + B.P if x1 + B.P < 2 ** 381 else B.P))),
           ("sig_x_c1_eq_p", bytes(g2_bytes(x0, B.P))),
           ("sig_x_c0_ge_p", bytes(g2_bytes(x0 + B.P if x0 + B.P < 2 ** 384 else B.P, x1, sig[0] & 0xE0))),
           ("sig_x_c0_all_ones", bytes(g2_bytes((1 << 384) - 1, x1, sig[0] & 0xE0))),
           ("sig_no_sqrt", no_sqrt_x_g2(r))]
    nc = bytearray(sig)
    nc[0] &= 0x7F
    out.append(("sig_uncompressed_flag", bytes(nc)))
    out.append(("sig_noncanonical_infinity_low", bytes([0xC0]) + bytes(94) + b"\x01"))
    out.append(("sig_noncanonical_infinity_c0", bytes([0xC0]) + bytes(47) + b"\x80" + bytes(47)))
    out.append(("sig_noncanonical_infinity_top", bytes([0xC1]) + bytes(95)))
    neg = bytearray(sig)
    neg[0] ^= 0x20
    out.append(("sig_sign_bit_flipped", bytes(neg)))
    return out


def main():
    cases = []
    # a 4-of-3 cluster for one validator (C1 shape)
    secret = rand_sk()
    coeffs = [rng.randrange(B.R) for _ in range(2)]
    shares = B.threshold_split(secret, 4, 3, coeffs)
    pubshares = {i: B.secret_to_public_key(s) for i, s in shares.items()}
    msg = hashlib.sha256(b"attestation-root").digest()
    parts = {i: B.sign(s, msg) for i, s in shares.items()}
    dv_pk = B.secret_to_public_key(secret)

    def add_verify(name, pk, m, sig, expect=None):
        st = B.verify(pk, m, sig)
        if expect is not None:
            assert st == expect, (name, st, expect)
        cases.append({"name": name, "pk": pk.hex(), "msg": m.hex(), "sig": sig.hex(), "status": st})

    for i in range(1, 5):
        add_verify(f"valid_share_{i}", pubshares[i], msg, parts[i], B.ST_OK)
    add_verify("wrong_message", pubshares[1], hashlib.sha256(b"other").digest(), parts[1], B.ST_NOT_VERIFIED)
    add_verify("wrong_share_index", pubshares[2], msg, parts[1], B.ST_NOT_VERIFIED)
    add_verify("random_96_bytes", pubshares[1], msg, bytes(rng.randrange(256) for _ in range(96)))
    add_verify("all_zero_signature", pubshares[1], msg, bytes(96), B.ST_BAD_SIGNATURE)
    add_verify("off_subgroup_sig", pubshares[1], msg, off_subgroup_g2(), B.ST_BAD_SIGNATURE)
    add_verify("infinity_sig", pubshares[1], msg, bytes([0xC0]) + bytes(95), B.ST_NOT_VERIFIED)
    add_verify("infinity_pk", bytes([0xC0]) + bytes(47), msg, bytes([0xC0]) + bytes(95), B.ST_NOT_VERIFIED)
    add_verify("pk_x_ge_p", bytes([0x80 | 0x1A]) + bytes([0xFF]) * 47, msg, parts[1], B.ST_BAD_PUBKEY)
    add_verify("pk_no_sqrt", no_sqrt_x_g1(), msg, parts[1], B.ST_BAD_PUBKEY)
    nc = bytearray(pubshares[1])
    nc[0] &= 0x7F
    add_verify("pk_uncompressed_flag", bytes(nc), msg, parts[1], B.ST_BAD_PUBKEY)
    add_verify("pk_off_subgroup", off_subgroup_g1(), msg, parts[1], B.ST_BAD_PUBKEY)
    add_verify("pk_noncanonical_infinity", bytes([0xC0]) + bytes(46) + b"\x01", msg, parts[1], B.ST_BAD_PUBKEY)
    add_verify("sig_infinity_with_sign_bit", pubshares[1], msg, bytes([0xE0]) + bytes(95), B.ST_BAD_SIGNATURE)
    hello = b"hello obol!"
    add_verify("hello_obol_dv", dv_pk, hello, B.sign(secret, hello), B.ST_OK)
    add_verify("empty_message", dv_pk, b"", B.sign(secret, b""), B.ST_OK)
    long_msg = bytes(rng.randrange(256) for _ in range(300))
    add_verify("long_message", pubshares[3], long_msg, B.sign(shares[3], long_msg), B.ST_OK)
    # G2-side non-canonical encodings (their own RNG stream: the cases above stay as they were)
    rng2 = random.Random(0x6253_4947)
    g2_rejects = g2_encoding_rejects(parts[1], rng2)
    for name, sig in g2_rejects:
        add_verify(name, pubshares[1], msg, sig,
                   B.ST_NOT_VERIFIED if name == "sig_sign_bit_flipped" else B.ST_BAD_SIGNATURE)

    # threshold aggregate
    ta = []

    def add_ta(name, group):
        st, out = B.threshold_aggregate(group)
        ta.append({"name": name, "partials": {str(k): v.hex() for k, v in group.items()}, "status": st,
                   "out": out.hex()})
        return st, out

    st, out = add_ta("t_of_n_123", {i: parts[i] for i in (1, 2, 3)})
    assert st == 0 and out == B.sign(secret, msg)
    st, out = add_ta("t_of_n_234", {i: parts[i] for i in (2, 3, 4)})
    assert out == B.sign(secret, msg)
    add_ta("all_n_1234", {i: parts[i] for i in (1, 2, 3, 4)})
    add_ta("k1", {3: parts[3]})
    add_ta("below_threshold_12", {i: parts[i] for i in (1, 2)})
    add_ta("index_zero", {0: parts[1], 2: parts[2], 3: parts[3]})
    add_ta("negative_index", {-3: parts[1], 2: parts[2], 3: parts[3]})
    add_ta("bad_partial", {1: parts[1], 2: bytes(96), 3: parts[3]})
    add_ta("off_subgroup_partial", {1: parts[1], 2: off_subgroup_g2(), 3: parts[3]})
    add_ta("empty", {})
    # 10-of-7 cluster
    secret7 = rand_sk()
    sh7 = B.threshold_split(secret7, 10, 7, [rng.randrange(B.R) for _ in range(6)])
    msg7 = hashlib.sha256(b"c3").digest()
    p7 = {i: B.sign(sh7[i], msg7) for i in (2, 3, 5, 7, 8, 9, 10)}
    st, out = add_ta("t7_of_10", p7)
    assert out == B.sign(secret7, msg7)
    # an undecodable member of every G2-side encoding class (herumi.go:262-268, via Sign.Deserialize)
    for name, sig in g2_rejects:
        if name == "sig_sign_bit_flipped":  # decodes: a wrong (but valid) aggregate, status OK
            st, out = add_ta("member_" + name, {1: parts[1], 2: sig, 3: parts[3]})
            assert st == B.ST_OK and out != B.sign(secret, msg)
            continue
        st, _ = add_ta("member_" + name, {1: parts[1], 2: sig, 3: parts[3]})
        assert st == B.ST_BAD_SIGNATURE, name

    # aggregate + verify_aggregate (tbls_test.go:129-167 shape)
    agg_cases = []
    sks = [rand_sk() for _ in range(10)]
    pks = [B.secret_to_public_key(s) for s in sks]
    sigs = [B.sign(s, hello) for s in sks]
    st, aggsig = B.aggregate(sigs)
    agg_cases.append({"name": "ten_keys", "sigs": [s.hex() for s in sigs], "status": st, "out": aggsig.hex()})
    st0, empty = B.aggregate([])
    agg_cases.append({"name": "empty", "sigs": [], "status": st0, "out": empty.hex()})
    agg_cases.append({"name": "bad_member", "sigs": [sigs[0].hex(), bytes(96).hex()], "status": B.ST_BAD_SIGNATURE,
                      "out": bytes(96).hex()})
    va = []
    va.append({"name": "ten_keys", "pks": [p.hex() for p in pks], "sig": aggsig.hex(), "msg": hello.hex(),
               "status": B.verify_aggregate(pks, aggsig, hello)})
    va.append({"name": "wrong_msg", "pks": [p.hex() for p in pks], "sig": aggsig.hex(), "msg": msg.hex(),
               "status": B.verify_aggregate(pks, aggsig, msg)})
    va.append({"name": "missing_key", "pks": [p.hex() for p in pks[1:]], "sig": aggsig.hex(), "msg": hello.hex(),
               "status": B.verify_aggregate(pks[1:], aggsig, hello)})
    va.append({"name": "no_keys", "pks": [], "sig": aggsig.hex(), "msg": hello.hex(),
               "status": B.verify_aggregate([], aggsig, hello)})
    va.append({"name": "bad_pk", "pks": [pks[0].hex(), off_subgroup_g1().hex()], "sig": aggsig.hex(),
               "msg": hello.hex(), "status": B.verify_aggregate([pks[0], off_subgroup_g1()], aggsig, hello)})

    out = {"generator": "tests/golden/make_fixtures.py (oracle/bls12381.py)",
           "cluster": {"secret": secret.hex(), "shares": {str(k): v.hex() for k, v in shares.items()},
                       "pubshares": {str(k): v.hex() for k, v in pubshares.items()}, "dv_pk": dv_pk.hex(),
                       "msg": msg.hex()},
           "verify": cases, "threshold_aggregate": ta, "aggregate": agg_cases, "verify_aggregate": va}
    with open(os.path.join(HERE, "fixtures_small.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote fixtures_small.json:", len(cases), "verify,", len(ta), "TA,", len(agg_cases), "agg,", len(va), "VA")


if __name__ == "__main__":
    main()
