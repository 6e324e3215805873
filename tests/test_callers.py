"""The host mirrors of charon's call sites (charon_amd/callers.py): one batch call per site, the
reference's first-error-aborts semantics and error strings.

CPU: against an oracle-backed stand-in implementation (test infrastructure), tiny inputs.
GPU (-m gpu): the same flows through the MI355X library (charon_amd.tbls.HIPBLS).
"""
import hashlib

import pytest

from charon_amd import callers
from charon_amd.callers import CallerError, ParSig
from oracle import bls12381 as B


class OracleImpl:
    """The batch methods of tbls.HIPBLS, restated with the oracle (CPU, test-only)."""

    def verify_batch(self, pks, msgs, sigs):
        return [B.verify(p, m, s) for p, m, s in zip(pks, msgs, sigs)]

    def threshold_aggregate_batch(self, groups):
        res = [B.threshold_aggregate(dict(g)) for g in groups]
        return [o for _, o in res], [s for s, _ in res]

    def verify_aggregate_batch(self, pk_groups, sigs, msgs):
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
    parts = {i: sign(s, root) for i, s in shares.items()}
    # parsigex: a peer's set with one entry, valid
    callers.parsigex_verify_set(impl, {dv: pubshares}, [(dv, ParSig(2, root, parts[2]))])
    # wrong message -> the reference's wrapped error chain
    with pytest.raises(CallerError, match="invalid partial signature: invalid signature: signature not verified"):
        callers.parsigex_verify_set(impl, {dv: pubshares}, [(dv, ParSig(2, hashlib.sha256(b"x").digest(), parts[2]))])
    with pytest.raises(CallerError, match="invalid shareIdx"):
        callers.parsigex_verify_set(impl, {dv: pubshares}, [(dv, ParSig(9, root, parts[2]))])
    with pytest.raises(CallerError, match="no signature found"):
        callers.parsigex_verify_set(impl, {dv: pubshares}, [(dv, ParSig(2, root, bytes(96)))])
    # sigagg: t partials -> the DV signature, verified under the DV key
    out = callers.sigagg_aggregate(impl, 3, {dv: dv}, {dv: [ParSig(i, root, parts[i]) for i in (1, 2, 3)]})
    assert out[dv] == sign(secret, root)
    with pytest.raises(CallerError, match="require threshold signatures"):
        callers.sigagg_aggregate(impl, 3, {dv: dv}, {dv: [ParSig(1, root, parts[1])]})
    with pytest.raises(CallerError, match="number of partial signatures less than threshold"):
        callers.sigagg_aggregate(impl, 3, {dv: dv}, {dv: [ParSig(1, root, parts[1])] * 3})
    with pytest.raises(CallerError, match="threshold aggregate: invalid signature: signature not verified"):
        callers.sigagg_aggregate(impl, 3, {dv: dv}, {dv: [ParSig(1, root, parts[1]), ParSig(2, root, parts[2]),
                                                           ParSig(3, root, parts[4])]})
    # exit: share 2 missing, threshold of the rest
    assert callers.exit_aggregate(impl, [parts[1], None, parts[3], parts[4]]) == sign(secret, root)
    # DKG deposit data: verify + aggregate + verify
    got = callers.dkg_agg_deposit_data(impl, {dv: pubshares}, {dv: [ParSig(i, root, parts[i]) for i in (1, 2, 4)]})
    assert got[dv] == sign(secret, root)
    with pytest.raises(CallerError, match="invalid deposit data partial signature from peer"):
        callers.dkg_agg_deposit_data(impl, {dv: pubshares}, {dv: [ParSig(1, root, parts[2])]})
    # lock: VerifyAggregate over the public shares
    lock_hash = hashlib.sha256(b"lock").digest()
    agg = B.aggregate([sign(s, lock_hash) for s in shares.values()])[1]
    callers.lock_verify_signatures(impl, list(pubshares.values()), agg, lock_hash)
    with pytest.raises(CallerError, match="verify lock signature aggregate: signature verification failed"):
        callers.lock_verify_signatures(impl, list(pubshares.values())[:3], agg, lock_hash)


@pytest.mark.slow
def test_caller_flows_oracle():
    _flows(OracleImpl(), B.sign, B.secret_to_public_key)


@pytest.mark.gpu
def test_caller_flows_gpu(hipbls):
    _flows(hipbls, hipbls.sign, hipbls.secret_to_public_key)
