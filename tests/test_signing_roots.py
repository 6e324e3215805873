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
