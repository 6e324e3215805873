"""Signing roots on the GPU (charon_amd/csrc/roots.hip) against the oracle's SSZ restatement.

The SSZ primitives of oracle/ssz.py (merkleize, uint64 / bytes32 leaves, SigningData, domains)
are pinned by the reference's Sign KATs (registration and deposit signatures byte-exact,
tests/test_oracle_kat.py); the AttestationData input is the reference's own SSZ fixture
(core/testdata/TestSSZSerialisation_AttestationData.ssz.golden, cross-checked against its JSON
twin by tests/golden/make_kats.py).  No reference file states an attestation root, so the
container layout (consensus-specs AttestationData) is the spec's, not a vector's.
"""
import hashlib
import random

import pytest

from oracle import ssz


def test_attestation_fixture_oracle(kats):
    a = kats["attestation_data"]
    data = bytes.fromhex(a["ssz"])
    assert ssz.attestation_data_root(data).hex() == a["htr_oracle"]
    # the container rule reproduces the pinned registration root shape: 5 leaves padded to 8
    slot, index, bbr, (se, sr), (te, tr) = ssz.parse_attestation_data(data)
    leaves = [ssz.htr_uint64(slot), ssz.htr_uint64(index), bbr, ssz.checkpoint_root(se, sr),
              ssz.checkpoint_root(te, tr)] + [bytes(32)] * 3
    h = lambda x, y: hashlib.sha256(x + y).digest()  # noqa: E731
    l1 = [h(leaves[i], leaves[i + 1]) for i in range(0, 8, 2)]
    assert h(h(l1[0], l1[1]), h(l1[2], l1[3])).hex() == a["htr_oracle"]


def _random_data(rng, n):
    out = []
    for _ in range(n):
        out.append(rng.randrange(2 ** 64).to_bytes(8, "little") + rng.randrange(2 ** 64).to_bytes(8, "little") +
                   rng.randbytes(32) + rng.randrange(2 ** 64).to_bytes(8, "little") + rng.randbytes(32) +
                   rng.randrange(2 ** 64).to_bytes(8, "little") + rng.randbytes(32))
    return out


@pytest.mark.gpu
def test_attestation_roots_gpu(kats, hipbls):
    from charon_amd import signing_roots as sr
    rng = random.Random(11)
    domains = [ssz.compute_domain(ssz.DOMAIN_BEACON_ATTESTER, v, rng.randbytes(32))
               for v in (bytes.fromhex("00000000"), bytes.fromhex("04017000"), bytes.fromhex("05000000"))]
    data = [bytes.fromhex(kats["attestation_data"]["ssz"])] + _random_data(rng, 1000)
    idx = [rng.randrange(3) for _ in data]
    got = sr.attestation_signing_roots(data, domains, idx)
    for i in list(range(40)) + [999, 1000]:
        assert got[i] == ssz.attestation_signing_root(data[i], domains[idx[i]]), i
    # object-root entry point: the same roots from the oracle's HTRs
    objs = [ssz.attestation_data_root(d) for d in data[:64]]
    assert sr.signing_roots(objs, domains, idx[:64]) == got[:64]
    # one shared domain (dom_idx omitted)
    assert sr.attestation_signing_roots(data[:5], domains[:1]) == \
        [ssz.attestation_signing_root(d, domains[0]) for d in data[:5]]
    assert sr.attestation_signing_roots([], domains) == []


@pytest.mark.gpu
def test_attestation_roots_device_feed_verify(kats, hipbls):
    """Roots computed on device feed signing and verification: sign over oracle roots, verify
    against roots the GPU derived from the same AttestationData."""
    from charon_amd import signing_roots as sr
    rng = random.Random(12)
    dom = [ssz.compute_domain(ssz.DOMAIN_BEACON_ATTESTER, bytes.fromhex("05000000"))]
    data = _random_data(rng, 16)
    keys = [hipbls.generate_secret_key() for _ in data]
    sigs = hipbls.sign_batch(keys, [ssz.attestation_signing_root(d, dom[0]) for d in data])
    roots = sr.attestation_signing_roots(data, dom)
    pks = [hipbls.secret_to_public_key(k) for k in keys]
    assert hipbls.verify_batch(pks, roots, sigs) == [0] * len(data)


def test_signing_roots_bad_input():
    from charon_amd import signing_roots as sr
    from charon_amd.tbls import TblsError
    with pytest.raises(TblsError):
        sr.attestation_signing_roots([bytes(127)], [bytes(32)])
    with pytest.raises(TblsError):
        sr.signing_roots([bytes(32)], [bytes(31)])


# ---- the other duty types (core/signeddata.go MessageRoot; hbls_duty_signing_roots)
_ORACLE_ROOT = {1: ssz.aggregate_and_proof_root, 2: ssz.contribution_and_proof_root,
                3: lambda b: ssz.sync_selection_root(int.from_bytes(b[:8], "little"), int.from_bytes(b[8:], "little")),
                4: lambda b: ssz.slot_root(int.from_bytes(b, "little")), 5: lambda b: b,
                6: ssz.validator_registration_ssz_root, 7: ssz.voluntary_exit_root,
                8: lambda b: ssz.epoch_root(int.from_bytes(b, "little")), 9: ssz.block_header_root}


def test_duty_fixtures_oracle(kats):
    """the oracle's object roots of the reference's duty goldens (committed by make_kats.py, each
    SSZ golden cross-checked against its JSON twin there) recompute; bitlist edge cases"""
    assert {k["name"] for k in kats["duty_roots"]} >= {"SignedAggregateAndProof", "SignedSyncContributionAndProof",
                                                       "SyncContributionAndProof", "BeaconCommitteeSelection",
                                                       "SignedSyncMessage", "VersionedSignedValidatorRegistration",
                                                       "SignedVoluntaryExit", "SignedRandao"}
    for k in kats["duty_roots"]:
        assert _ORACLE_ROOT[k["kind"]](bytes.fromhex(k["ssz"])).hex() == k["object_root"], k["name"]
    # the registration object's signing root under the builder domain is the pinned registration
    # KAT message (its teku signature verifies over it, tests/test_oracle_kat.py)
    reg = next(k for k in kats["duty_roots"] if k["kind"] == 6)
    assert ssz.signing_root(bytes.fromhex(reg["object_root"]),
                            bytes.fromhex(kats["registration"]["domain"])).hex() == kats["registration"]["msg"]
    # a block header's root: the 5-field container (8 leaves, 3 zero)
    hdr = bytes(range(112))
    h = lambda x, y: hashlib.sha256(x + y).digest()  # noqa: E731
    z = bytes(32)
    leaves = [hdr[0:8] + bytes(24), hdr[8:16] + bytes(24), hdr[16:48], hdr[48:80], hdr[80:112]]
    assert ssz.block_header_root(hdr) == h(h(h(leaves[0], leaves[1]), h(leaves[2], leaves[3])),
                                           h(h(leaves[4], z), h(z, z)))
    # Bitlist[2048]: empty (delimiter only), one bit, a full chunk, the maximum
    h = lambda x, y: hashlib.sha256(x + y).digest()  # noqa: E731
    z = bytes(32)
    zero8 = ssz.merkleize([z] * 8)
    assert ssz.bitlist_root(b"\x01", 2048) == h(zero8, bytes(32))
    assert ssz.bitlist_root(b"\x03", 2048) == h(ssz.merkleize([b"\x01" + bytes(31)] + [z] * 7), (1).to_bytes(32, "little"))
    full = bytes([0xff] * 256) + b"\x01"
    assert ssz.bitlist_root(full, 2048) == h(ssz.merkleize([bytes([0xff] * 32)] * 8), (2048).to_bytes(32, "little"))
    with pytest.raises(AssertionError):
        ssz.bitlist_root(bytes([0xff] * 256) + b"\x03", 2048)  # 2049 bits


def _aggregate_and_proof(rng, nbits):
    bits = rng.getrandbits(nbits) if nbits else 0
    bl = (bits | (1 << nbits)).to_bytes(nbits // 8 + 1, "little")
    att = (228).to_bytes(4, "little") + _random_data(rng, 1)[0] + rng.randbytes(96) + bl
    return rng.randrange(2 ** 64).to_bytes(8, "little") + (108).to_bytes(4, "little") + rng.randbytes(96) + att


@pytest.mark.gpu
def test_duty_roots_gpu(kats, hipbls):
    """device object and signing roots of every duty kind equal the oracle's: the reference's
    goldens, random objects (bitlists of 0..2048 bits), one shared and per-item domains, and
    malformed objects rejected with HBLS_BAD_INPUT and a zero root"""
    from charon_amd import signing_roots as sr
    rng = random.Random(12)
    domains = [rng.randbytes(32) for _ in range(3)]
    gold = {}
    for k in kats["duty_roots"]:
        gold.setdefault(k["kind"], []).append(bytes.fromhex(k["ssz"]))
    objs = {1: gold[1] + [_aggregate_and_proof(rng, nb) for nb in (0, 1, 7, 8, 9, 255, 256, 257, 1000, 2047, 2048)],
            2: gold[2] + [rng.randbytes(264) for _ in range(20)],
            3: gold[3] + [rng.randbytes(16) for _ in range(20)],
            4: gold[4] + [rng.randbytes(8) for _ in range(20)],
            5: gold[5] + [rng.randbytes(32) for _ in range(20)],
            6: gold[6] + [rng.randbytes(84) for _ in range(20)],
            7: gold[7] + [rng.randbytes(16) for _ in range(20)],
            8: gold[8] + [rng.randbytes(8) for _ in range(20)],
            9: [rng.randbytes(112) for _ in range(20)]}
    for kind, obs in objs.items():
        idx = [rng.randrange(3) for _ in obs]
        roots, st = sr.duty_signing_roots(kind, obs, domains, idx)
        assert st == [0] * len(obs), kind
        for o, r, i in zip(obs, roots, idx):
            assert r == ssz.signing_root(_ORACLE_ROOT[kind](o), domains[i]), kind
        roots1, _ = sr.duty_signing_roots(kind, obs[:3], domains[:1])
        assert roots1 == [ssz.signing_root(_ORACLE_ROOT[kind](o), domains[0]) for o in obs[:3]]
    good = _aggregate_and_proof(rng, 20)
    bad = [good[:200],                                            # truncated
           good[:8] + (100).to_bytes(4, "little") + good[12:],    # wrong offset
           good[:-1] + b"\x00",                                   # no delimiter
           _aggregate_and_proof(rng, 2048)[:-1] + b"\x03"]        # 2049 bits
    roots, st = sr.duty_signing_roots(1, [good] + bad, domains)
    assert st == [0, 6, 6, 6, 6] and all(r == bytes(32) for r in roots[1:])
    roots, st = sr.duty_signing_roots(2, [rng.randbytes(263)], domains)
    assert st == [6] and roots == [bytes(32)]
    for kind, size in ((6, 84), (7, 16), (8, 8), (9, 112)):
        roots, st = sr.duty_signing_roots(kind, [rng.randbytes(size - 1), rng.randbytes(size + 1)], domains)
        assert st == [6, 6] and roots == [bytes(32)] * 2, kind


@pytest.mark.gpu
def test_registration_root_on_device_verifies_teku_signature(kats, hipbls):
    """The teku registration (eth2util/signing/signing_test.go) through the device: its SSZ object
    rooted under the builder domain by hbls_duty_signing_roots kind 6 is the message the teku
    signature verifies over -- the reference's own vector pins the device's registration root."""
    from charon_amd import signing_roots as sr
    r = kats["registration"]
    obj = bytes.fromhex(next(k for k in kats["duty_roots"] if k["kind"] == 6)["ssz"])
    roots, st = sr.duty_signing_roots(sr.VALIDATOR_REGISTRATION, [obj], [bytes.fromhex(r["domain"])])
    assert st == [0] and roots[0].hex() == r["msg"]
    pk = hipbls.secret_to_public_key(bytes.fromhex(r["sk"]))
    assert hipbls.verify_batch([pk], roots, [bytes.fromhex(r["sig"])]) == [0]
