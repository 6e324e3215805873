"""The host mirrors of charon's call sites (charon_amd/callers.py): batch calls per site, the
reference's error strings, and the error the reference's per-item loop returns first.

CPU: against an oracle-backed stand-in implementation (test infrastructure), tiny inputs.
GPU (-m gpu): the same flows through the MI355X library (charon_amd.tbls.HIPBLS).
"""
import hashlib

import pytest

from charon_amd import callers
from charon_amd.callers import CallerError, ParSig
from oracle import bls12381 as B


class OracleImpl:
    """The batch methods of tbls.HIPBLS, restated with the oracle (CPU, test-only); counts calls."""

    def __init__(self):
        self.calls = []

    def verify_batch(self, pks, msgs, sigs):
        self.calls.append(("verify", len(pks)))
        return [B.verify(p, m, s) for p, m, s in zip(pks, msgs, sigs)]

    def threshold_aggregate_batch(self, groups):
        self.calls.append(("ta", len(groups)))
        res = [B.threshold_aggregate(dict(g)) for g in groups]
        return [o for _, o in res], [s for s, _ in res]

    def aggregate_batch(self, groups):
        self.calls.append(("aggregate", len(groups)))
        res = [B.aggregate(list(g)) for g in groups]
        return [o for _, o in res], [s for s, _ in res]

    def verify_aggregate_batch(self, pk_groups, sigs, msgs):
        self.calls.append(("verify_aggregate", len(pk_groups)))
        return [B.verify_aggregate(list(p), s, m) for p, s, m in zip(pk_groups, sigs, msgs)]


def _cluster(n=4, t=3, seed=b"callers"):
    secret = (int.from_bytes(hashlib.sha256(seed).digest(), "big") % B.R).to_bytes(32, "big")
    coeffs = [int.from_bytes(hashlib.sha256(seed + bytes([k])).digest(), "big") % B.R for k in range(t - 1)]
    shares = B.threshold_split(secret, n, t, coeffs)
    return secret, shares


def _flows(impl, sign, pub):
    secret, shares = _cluster()
    dv = pub(secret)
    pubshares = {i: pub(s) for i, s in shares.items()}
    root = hashlib.sha256(b"attestation data root").digest()
    other = hashlib.sha256(b"x").digest()
    parts = {i: sign(s, root) for i, s in shares.items()}
    wrong = sign(shares[2], other)  # share 2's partial over another message
    W = "invalid partial signature"

    # --- parsigex (parsigex.go:93-98, NewEth2Verifier :145-170)
    callers.parsigex_verify_set(impl, {dv: pubshares}, [(dv, ParSig(2, root, parts[2]))])
    with pytest.raises(CallerError, match=f"^{W}: invalid signature: signature not verified$"):
        callers.parsigex_verify_set(impl, {dv: pubshares}, [(dv, ParSig(2, other, parts[2]))])
    with pytest.raises(CallerError, match=f"^{W}: invalid shareIdx$"):
        callers.parsigex_verify_set(impl, {dv: pubshares}, [(dv, ParSig(9, root, parts[2]))])
    with pytest.raises(CallerError, match=f"^{W}: invalid signature: no signature found$"):
        callers.parsigex_verify_set(impl, {dv: pubshares}, [(dv, ParSig(2, root, bytes(96)))])
    with pytest.raises(CallerError, match=f"^{W}: unknown pubkey, not part of cluster lock$"):
        callers.parsigex_verify_set(impl, {dv: pubshares}, [(b"\x01" * 48, ParSig(2, root, parts[2]))])
    # first error in set order: a wrong signature before a bad share index wins, and vice versa
    dv2 = pub(shares[1])
    ps2 = {dv: pubshares, dv2: pubshares}
    with pytest.raises(CallerError, match="signature not verified"):
        callers.parsigex_verify_set(impl, ps2, [(dv, ParSig(2, other, parts[2])), (dv2, ParSig(9, root, parts[2]))])
    with pytest.raises(CallerError, match="invalid shareIdx"):
        callers.parsigex_verify_set(impl, ps2, [(dv2, ParSig(9, root, parts[2])), (dv, ParSig(2, other, parts[2]))])

    # --- sigagg: t partials -> the DV signature, verified under the DV key (sigagg.go:48-144)
    out = callers.sigagg_aggregate(impl, 3, {dv: dv}, {dv: [ParSig(i, root, parts[i]) for i in (1, 2, 3)]})
    assert out[dv] == sign(secret, root)
    with pytest.raises(CallerError, match="^threshold aggregate: require threshold signatures$"):
        callers.sigagg_aggregate(impl, 3, {dv: dv}, {dv: [ParSig(1, root, parts[1])]})
    with pytest.raises(CallerError, match="^threshold aggregate: number of partial signatures less than threshold$"):
        callers.sigagg_aggregate(impl, 3, {dv: dv}, {dv: [ParSig(1, root, parts[1])] * 3})
    # a wrong member gives a wrong aggregate: NewVerifier's wrapped error (sigagg.go:139)
    with pytest.raises(CallerError, match="^threshold aggregate: aggregate signature verification failed: "
                                          "signature not verified$"):
        callers.sigagg_aggregate(impl, 3, {dv: dv}, {dv: [ParSig(1, root, parts[1]), ParSig(2, root, parts[2]),
                                                           ParSig(3, root, parts[4])]})
    with pytest.raises(CallerError, match="^threshold aggregate: cannot unmarshal signature into Herumi signature$"):
        callers.sigagg_aggregate(impl, 3, {dv: dv}, {dv: [ParSig(1, root, parts[1]), ParSig(2, root, parts[2]),
                                                           ParSig(3, root, b"\x11" * 96)]})
    # validator order: the first validator's TA failure beats the second's pre-check failure
    with pytest.raises(CallerError, match="cannot unmarshal signature"):
        callers.sigagg_aggregate(impl, 3, {dv: dv, dv2: dv2},
                                 {dv: [ParSig(1, root, parts[1]), ParSig(2, root, parts[2]), ParSig(3, root, b"\x11" * 96)],
                                  dv2: [ParSig(1, root, parts[1])]})
    with pytest.raises(CallerError, match="require threshold signatures"):
        callers.sigagg_aggregate(impl, 3, {dv: dv, dv2: dv2},
                                 {dv2: [ParSig(1, root, parts[1])],
                                  dv: [ParSig(1, root, parts[1]), ParSig(2, root, parts[2]), ParSig(3, root, b"\x11" * 96)]})

    # --- validatorapi (validatorapi.go:284-306, verifyPartialSig :1213-1229): first attestation's error
    callers.validatorapi_submit(impl, {dv: pubshares[2]}, [(dv, root, parts[2])])
    with pytest.raises(CallerError, match="^signature not verified$"):
        callers.validatorapi_submit(impl, {dv: pubshares[2]}, [(dv, root, parts[2]), (dv, other, parts[2])])
    with pytest.raises(CallerError, match="^no signature found$"):
        callers.validatorapi_submit(impl, {dv: pubshares[2]}, [(dv, root, bytes(96)), (dv, other, parts[2])])
    with pytest.raises(CallerError, match="^signature not verified$"):  # the wrong signature comes first
        callers.validatorapi_submit(impl, {dv: pubshares[2]}, [(dv, other, parts[2]), (dv2, root, parts[2])])
    with pytest.raises(CallerError, match="^unknown public key$"):
        callers.validatorapi_submit(impl, {dv: pubshares[2]}, [(dv2, root, parts[2]), (dv, other, parts[2])])

    # --- exit: share 2 missing, threshold of the rest (exit.go:165-194)
    assert callers.exit_aggregate(impl, [parts[1], None, parts[3], parts[4]]) == sign(secret, root)
    with pytest.raises(CallerError, match="^partial signatures threshold aggregate: cannot combine signatures$"):
        callers.exit_aggregate(impl, [None, None, None, None])
    full = callers.exit_aggregate_batch(impl, [("0xa", [parts[1], parts[2], None, parts[4]]),
                                               ("0xb", [None, parts[2], parts[3], parts[4]])])
    assert full == [sign(secret, root)] * 2
    with pytest.raises(CallerError, match="^load full exit data from Obol API: partial signatures threshold "
                                          "aggregate: cannot unmarshal signature into Herumi signature$"):
        callers.exit_aggregate_batch(impl, [("0xa", [parts[1], parts[2], None, parts[4]]),
                                            ("0xb", [b"\x11" * 96, parts[2], parts[3], None])])
    # validator 0's aggregation error comes before validator 1's length error (exit_fetch.go:122-132)
    with pytest.raises(CallerError, match="^load full exit data from Obol API: partial signatures threshold "
                                          "aggregate: cannot unmarshal signature into Herumi signature$"):
        callers.exit_aggregate_batch(impl, [("0xa", [b"\x11" * 96, parts[2], parts[3], None]),
                                            ("0xb", [parts[1], parts[2][:95], parts[3], None])])
    # ... and a length error of an earlier validator before a later aggregation error
    with pytest.raises(CallerError, match="^load full exit data from Obol API: invalid partial signature: "
                                          "data is not of the correct length$"):
        callers.exit_aggregate_batch(impl, [("0xa", [parts[1], parts[2][:95], parts[3], None]),
                                            ("0xb", [b"\x11" * 96, parts[2], parts[3], None])])

    # --- DKG deposit data / registrations: verify + aggregate + verify per DV (dkg.go:820-984)
    roots = {dv: root}
    got = callers.dkg_agg_deposit_data(impl, {dv: pubshares}, {dv: [ParSig(i, root, parts[i]) for i in (1, 2, 4)]}, roots)
    assert got[dv] == sign(secret, root)
    with pytest.raises(CallerError, match="^invalid deposit data partial signature from peer$"):
        callers.dkg_agg_deposit_data(impl, {dv: pubshares}, {dv: [ParSig(1, root, parts[2])]}, roots)
    with pytest.raises(CallerError, match="^deposit message not found$"):
        callers.dkg_agg_deposit_data(impl, {dv: pubshares}, {dv: [ParSig(1, root, parts[1])]}, {})
    with pytest.raises(CallerError, match="^invalid pubshare$"):
        callers.dkg_agg_deposit_data(impl, {dv: pubshares}, {dv: [ParSig(7, root, parts[1])]}, roots)
    # a bad partial of share 1 is reported before the missing share 7 later in the same DV
    with pytest.raises(CallerError, match="^invalid deposit data partial signature from peer$"):
        callers.dkg_agg_deposit_data(impl, {dv: pubshares}, {dv: [ParSig(1, root, parts[2]), ParSig(7, root, parts[1])]},
                                     roots)
    got = callers.dkg_agg_validator_registrations(impl, {dv: pubshares},
                                                  {dv: [ParSig(i, root, parts[i]) for i in (2, 3, 4)]}, roots)
    assert got[dv] == sign(secret, root)
    with pytest.raises(CallerError, match="^invalid validator registration partial signature from peer$"):
        callers.dkg_agg_validator_registrations(impl, {dv: pubshares}, {dv: [ParSig(3, root, wrong)]}, roots)
    with pytest.raises(CallerError, match="^invalid pubkey in validator registrations partial signature from peer$"):
        callers.dkg_agg_validator_registrations(impl, {}, {dv: [ParSig(3, root, parts[3])]}, roots)
    # a wrong member set: the aggregate fails its own check (dkg.go:975-978)
    with pytest.raises(CallerError, match="^invalid validator registration aggregated signature: signature not verified$"):
        callers.dkg_agg_validator_registrations(impl, {dv: pubshares}, {dv: [ParSig(2, root, parts[2]),
                                                                            ParSig(3, root, parts[3])]}, roots)

    # --- DKG lock hash: every partial verified, one plain aggregate, VerifyAggregate (dkg.go:590-703)
    lock_hash = hashlib.sha256(b"lock").digest()
    lparts = {i: sign(s, lock_hash) for i, s in shares.items()}
    agg, pks = callers.dkg_agg_lock_hash_sig(impl, {dv: pubshares}, {dv: [ParSig(i, lock_hash, lparts[i]) for i in (1, 2, 3, 4)]},
                                             lock_hash)
    assert pks == [pubshares[i] for i in (1, 2, 3, 4)]
    callers.dkg_verify_lock_multisig(impl, pks, agg, lock_hash)
    with pytest.raises(CallerError, match="^verify multisignature: signature verification failed$"):
        callers.dkg_verify_lock_multisig(impl, pks[:3], agg, lock_hash)
    with pytest.raises(CallerError, match="^invalid lock hash partial signature from peer: signature not verified$"):
        callers.dkg_agg_lock_hash_sig(impl, {dv: pubshares}, {dv: [ParSig(1, lock_hash, lparts[2])]}, lock_hash)
    with pytest.raises(CallerError, match="^signature from bytes: data is not of the correct length$"):
        callers.dkg_agg_lock_hash_sig(impl, {dv: pubshares}, {dv: [ParSig(1, lock_hash, lparts[1][:95])]}, lock_hash)

    # --- lock: VerifyAggregate over the public shares (lock.go:185)
    agg = B.aggregate([sign(s, lock_hash) for s in shares.values()])[1]
    callers.lock_verify_signatures(impl, list(pubshares.values()), agg, lock_hash)
    with pytest.raises(CallerError, match="verify lock signature aggregate: signature verification failed"):
        callers.lock_verify_signatures(impl, list(pubshares.values())[:3], agg, lock_hash)


@pytest.mark.slow
def test_caller_flows_oracle():
    _flows(OracleImpl(), B.sign, B.secret_to_public_key)


def test_caller_batching_one_call_per_step():
    """The mirrors issue one batch call per step, not one per item (counted on the stand-in):
    a sigagg duty set of 3 validators is one ThresholdAggregate batch and one Verify batch."""
    impl = OracleImpl()
    secret, shares = _cluster(seed=b"batching")
    root = hashlib.sha256(b"r").digest()
    parts = {i: B.sign(s, root) for i, s in shares.items()}
    dv = B.secret_to_public_key(secret)
    sets = {dv + bytes([k]): [ParSig(i, root, parts[i]) for i in (1, 2, 3)] for k in range(3)}
    out = callers.sigagg_aggregate(impl, 3, {k: dv for k in sets}, sets)
    assert set(out.values()) == {B.sign(secret, root)}
    assert impl.calls == [("ta", 3), ("verify", 3)]


@pytest.mark.gpu
def test_caller_flows_gpu(hipbls):
    _flows(hipbls, hipbls.sign, hipbls.secret_to_public_key)
