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


# ---- the other duty types whose signing roots charon verifies in bulk (core/signeddata.go
# MessageRoot): SignedAggregateAndProof (:979, phase0.AggregateAndProof.HashTreeRoot),
# SignedSyncMessage (:1056, the beacon block root itself), SyncContributionAndProof (:1135,
# altair.SyncAggregatorSelectionData{slot, subcommittee_index}.HashTreeRoot),
# SignedSyncContributionAndProof (:1227, altair.ContributionAndProof.HashTreeRoot),
# BeaconCommitteeSelection (:852, eth2util.SlotHashRoot: the uint64 slot as one chunk).
MAX_VALIDATORS_PER_COMMITTEE = 2048
SYNC_SUBCOMMITTEE_SIZE = 128  # SYNC_COMMITTEE_SIZE / SYNC_COMMITTEE_SUBNET_COUNT (mainnet)


def mix_in_length(root: bytes, length: int) -> bytes:
    return _h(root, length.to_bytes(32, "little"))


def bitlist_root(b: bytes, limit: int) -> bytes:
    """hash_tree_root of an SSZ Bitlist[limit] from its encoding (delimiter bit after the last)."""
    assert len(b) >= 1 and b[-1] != 0, "bitlist without delimiter"
    nbits = 8 * (len(b) - 1) + b[-1].bit_length() - 1
    assert nbits <= limit
    v = int.from_bytes(b, "little") ^ (1 << nbits)  # drop the delimiter
    data = v.to_bytes((nbits + 7) // 8, "little") if nbits else b""
    chunks = [_chunk(data[i:i + 32]) for i in range(0, len(data), 32)]
    limit_chunks = (limit + 255) // 256
    layer = chunks + [bytes(32)] * (limit_chunks - len(chunks))
    return mix_in_length(merkleize(layer), nbits)


def signature_root(sig: bytes) -> bytes:
    assert len(sig) == 96
    return htr_bytes_fixed(sig)


def attestation_root(b: bytes) -> bytes:
    """phase0.Attestation{aggregation_bits Bitlist[2048], data AttestationData, signature}: the
    fixed part is the bits' offset, the 128-byte data and the 96-byte signature."""
    off = int.from_bytes(b[0:4], "little")
    assert off == 228 and len(b) > off
    return merkleize([bitlist_root(b[off:], MAX_VALIDATORS_PER_COMMITTEE), attestation_data_root(b[4:132]),
                      signature_root(b[132:228])])


def aggregate_and_proof_root(b: bytes) -> bytes:
    """phase0.AggregateAndProof{aggregator_index, aggregate Attestation, selection_proof}."""
    off = int.from_bytes(b[8:12], "little")
    assert off == 108 and len(b) > off
    return merkleize([htr_uint64(int.from_bytes(b[0:8], "little")), attestation_root(b[off:]),
                      signature_root(b[12:108])])


def sync_committee_contribution_root(b: bytes) -> bytes:
    """altair.SyncCommitteeContribution{slot, beacon_block_root, subcommittee_index,
    aggregation_bits Bitvector[128], signature}: 160 bytes."""
    assert len(b) == 160
    u = lambda o: int.from_bytes(b[o:o + 8], "little")  # noqa: E731
    return merkleize([htr_uint64(u(0)), b[8:40], htr_uint64(u(40)), htr_bytes_fixed(b[48:64]),
                      signature_root(b[64:160])])


def contribution_and_proof_root(b: bytes) -> bytes:
    """altair.ContributionAndProof{aggregator_index, contribution, selection_proof}: 264 bytes."""
    assert len(b) == 264
    return merkleize([htr_uint64(int.from_bytes(b[0:8], "little")), sync_committee_contribution_root(b[8:168]),
                      signature_root(b[168:264])])


def sync_selection_root(slot: int, subcommittee_index: int) -> bytes:
    """altair.SyncAggregatorSelectionData{slot, subcommittee_index}."""
    return merkleize([htr_uint64(slot), htr_uint64(subcommittee_index)])


def slot_root(slot: int) -> bytes:
    """eth2util.SlotHashRoot (eth2util/hash.go:13-30): one uint64 merkleized alone = its chunk."""
    return htr_uint64(slot)


def voluntary_exit_root(b: bytes) -> bytes:
    """phase0.VoluntaryExit{epoch, validator_index}: 16 bytes (core/signeddata.go:580)."""
    assert len(b) == 16
    return merkleize([htr_uint64(int.from_bytes(b[0:8], "little")), htr_uint64(int.from_bytes(b[8:16], "little"))])


def epoch_root(epoch: int) -> bytes:
    """eth2util.SignedEpoch.HashTreeRoot (eth2util/types.go:245-258): the epoch's uint64 chunk."""
    return htr_uint64(epoch)


def validator_registration_ssz_root(b: bytes) -> bytes:
    """v1.ValidatorRegistration from its 84-byte SSZ: fee_recipient(20) gas_limit timestamp pubkey(48)."""
    assert len(b) == 84
    return validator_registration_root(b[0:20], int.from_bytes(b[20:28], "little"), int.from_bytes(b[28:36], "little"),
                                       b[36:84])


def block_header_root(b: bytes) -> bytes:
    """phase0.BeaconBlockHeader{slot, proposer_index, parent_root, state_root, body_root}: 112
    bytes; a BeaconBlock's hash-tree-root equals its header's (body replaced by its root)."""
    assert len(b) == 112
    return merkleize([htr_uint64(int.from_bytes(b[0:8], "little")), htr_uint64(int.from_bytes(b[8:16], "little")),
                      b[16:48], b[48:80], b[80:112]])
