"""CPU oracle helper: the few SSZ hash-tree-roots charon uses to build 32-byte signing roots.

TEST INFRASTRUCTURE ONLY (used to re-derive the messages of the reference's known-answer
vectors).  Restates:
  * eth2util/signing/signing.go:63-77 (GetDataRoot: SigningData{object_root, domain})
  * eth2util/registration/registration.go:65-101 (DOMAIN_APPLICATION_BUILDER, genesis fork)
  * eth2util/deposit/deposit.go:131-170 (DOMAIN_DEPOSIT, genesis fork)
  * consensus-specs compute_domain / ForkData / ValidatorRegistration / DepositMessage SSZ.
"""

from __future__ import annotations

import hashlib


def _h(a: bytes, b: bytes) -> bytes:
    return hashlib.sha256(a + b).digest()


def _chunk(b: bytes) -> bytes:
    assert len(b) <= 32
    return b + bytes(32 - len(b))


def merkleize(chunks):
    n = 1
    while n < len(chunks):
        n *= 2
    layer = list(chunks) + [bytes(32)] * (n - len(chunks))
    while len(layer) > 1:
        layer = [_h(layer[i], layer[i + 1]) for i in range(0, len(layer), 2)]
    return layer[0]


def htr_bytes_fixed(b: bytes) -> bytes:
    """hash_tree_root of a fixed-size ByteVector."""
    chunks = [_chunk(b[i:i + 32]) for i in range(0, len(b), 32)] or [bytes(32)]
    return merkleize(chunks)


def htr_uint64(v: int) -> bytes:
    return _chunk(v.to_bytes(8, "little"))


def fork_data_root(version: bytes, genesis_validators_root: bytes = bytes(32)) -> bytes:
    return merkleize([_chunk(version), genesis_validators_root])


def compute_domain(domain_type: bytes, fork_version: bytes, gvr: bytes = bytes(32)) -> bytes:
    return domain_type + fork_data_root(fork_version, gvr)[:28]


def signing_root(object_root: bytes, domain: bytes) -> bytes:
    return merkleize([object_root, domain])


def validator_registration_root(fee_recipient: bytes, gas_limit: int, timestamp: int, pubkey: bytes) -> bytes:
    return merkleize([
        htr_bytes_fixed(fee_recipient),
        htr_uint64(gas_limit),
        htr_uint64(timestamp),
        htr_bytes_fixed(pubkey),
    ])


def deposit_message_root(pubkey: bytes, withdrawal_credentials: bytes, amount: int) -> bytes:
    return merkleize([htr_bytes_fixed(pubkey), htr_bytes_fixed(withdrawal_credentials), htr_uint64(amount)])


DOMAIN_APPLICATION_BUILDER = bytes.fromhex("00000001")
DOMAIN_DEPOSIT = bytes.fromhex("03000000")


# ---- attestations (the slot's hot message): core/signeddata.go Attestation.MessageRoot ->
# phase0.AttestationData.HashTreeRoot (go-eth2-client's generated SSZ, consensus-specs container
# AttestationData{slot, index, beacon_block_root, source: Checkpoint, target: Checkpoint}).
DOMAIN_BEACON_ATTESTER = bytes.fromhex("01000000")
ATTESTATION_DATA_SSZ_LEN = 128


def checkpoint_root(epoch: int, root: bytes) -> bytes:
    return merkleize([htr_uint64(epoch), root])


def parse_attestation_data(b: bytes):
    """SSZ bytes (fixed layout, 128 B) -> (slot, index, beacon_block_root, (src_epoch, src_root),
    (tgt_epoch, tgt_root))."""
    assert len(b) == ATTESTATION_DATA_SSZ_LEN
    u = lambda o: int.from_bytes(b[o:o + 8], "little")  # noqa: E731
    return u(0), u(8), b[16:48], (u(48), b[56:88]), (u(88), b[96:128])


def attestation_data_root(b: bytes) -> bytes:
    slot, index, bbr, (se, sr), (te, tr) = parse_attestation_data(b)
    return merkleize([htr_uint64(slot), htr_uint64(index), bbr, checkpoint_root(se, sr), checkpoint_root(te, tr)])


def attestation_signing_root(b: bytes, domain: bytes) -> bytes:
    """GetDataRoot (signing.go:63-77) of an attestation: SigningData{HTR(data), domain}."""
    return signing_root(attestation_data_root(b), domain)
