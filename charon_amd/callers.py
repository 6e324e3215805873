"""Host-side mirrors of charon's BLS call sites, switched to the batch entry points (SURVEY.md
§8(f)1 and §8(f)4).  Each function keeps the reference's first-error-aborts semantics and error
strings; only the per-item tbls calls are replaced by one batch call.  INTEGRATION.md §3 gives the
same changes as Go patches.

  parsigex_verify_set      core/parsigex/parsigex.go:93-98 + NewEth2Verifier :145-170
                           (+ eth2util/signing/signing.go:96-115 zero-signature check)
  sigagg_aggregate         core/sigagg/sigagg.go:48-81 + aggregate :83-122 (TA :105, verify :117)
  validatorapi_submit      core/validatorapi/validatorapi.go:284-306 + verifyPartialSig :1213-1229
  lock_verify_signatures   cluster/lock.go:151-197 (VerifyAggregate over every pubshare, :185)
  dkg_agg_deposit_data     dkg/dkg.go:820-899 (n x Verify + ThresholdAggregate + Verify per DV)
  exit_aggregate           app/obolapi/exit.go:165-194 (ThresholdAggregate of the exit partials)

`impl` is any object with the batch methods of charon_amd.tbls.HIPBLS (verify_batch,
threshold_aggregate_batch, verify_aggregate_batch).  Messages are the 32-byte signing roots the
callers compute (eth2util/signing.GetDataRoot), or roots computed on the GPU by
charon_amd.signing_roots.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Mapping, Optional, Sequence, Tuple

from .tbls import TblsError, _TA_ERR, _VERIFY_AGG_ERR, _VERIFY_ERR

OK = 0
ZERO_SIG = bytes(96)


class CallerError(TblsError):
    """The error a reference call site returns (wrapped message, as errors.Wrap prints it)."""


def _wrap(outer: str, inner: str) -> CallerError:
    return CallerError(f"{outer}: {inner}")


@dataclass
class ParSig:
    """core.ParSignedData reduced to what verification needs."""
    share_idx: int
    signing_root: bytes
    signature: bytes


def parsigex_verify_set(impl, pubshares_by_key: Mapping[bytes, Mapping[int, bytes]],
                        data_set: Sequence[Tuple[bytes, ParSig]]) -> None:
    """ParSigEx.handle's verification loop (parsigex.go:93-98) over a peer's whole set in one
    batch.  The first failing entry (in set order) aborts with the reference's error chain:
    "invalid partial signature: invalid signature: <tbls error>"."""
    pks, msgs, sigs = [], [], []
    for pubkey, ps in data_set:
        shares = pubshares_by_key.get(pubkey)
        if shares is None:
            raise _wrap("invalid partial signature", "unknown pubkey, not part of cluster lock")
        pubshare = shares.get(ps.share_idx)
        if pubshare is None:
            raise _wrap("invalid partial signature", "invalid shareIdx")
        if ps.signature == ZERO_SIG:  # signing.go:107-110, before tbls.Verify
            raise _wrap("invalid partial signature", "invalid signature: no signature found")
        pks.append(pubshare)
        msgs.append(ps.signing_root)
        sigs.append(ps.signature)
    st = impl.verify_batch(pks, msgs, sigs) if pks else []
    for s in st:
        if s != OK:
            raise _wrap("invalid partial signature", "invalid signature: " + _VERIFY_ERR.get(s, "signature not verified"))


def sigagg_aggregate(impl, threshold: int, dv_pubkeys: Mapping[bytes, bytes],
                     sets: Mapping[bytes, Sequence[ParSig]]) -> Dict[bytes, bytes]:
    """Aggregator.Aggregate (sigagg.go:48-81): every validator's partials threshold-aggregated in
    one batch, then every aggregate verified under its DV key in one batch (sigagg.go:117).  The
    first validator whose step fails aborts the duty set with "threshold aggregate: <error>"."""
    if not sets:
        raise CallerError("empty partial signed data set")
    keys = list(sets)
    groups = []
    for pk in keys:
        par = sets[pk]
        if len(par) < threshold:
            raise _wrap("threshold aggregate", "require threshold signatures")
        by_idx: Dict[int, bytes] = {}
        for ps in par:
            by_idx[ps.share_idx] = ps.signature
        if len(by_idx) < threshold:
            raise _wrap("threshold aggregate", "number of partial signatures less than threshold")
        groups.append(by_idx)
    outs, sts = impl.threshold_aggregate_batch(groups)
    for s in sts:
        if s != OK:
            raise _wrap("threshold aggregate", _TA_ERR.get(s, "cannot combine signatures"))
    roots = [sets[pk][0].signing_root for pk in keys]
    vst = impl.verify_batch([dv_pubkeys[pk] for pk in keys], roots, outs)
    for s in vst:
        if s != OK:
            raise _wrap("threshold aggregate", "invalid signature: " + _VERIFY_ERR.get(s, "signature not verified"))
    return dict(zip(keys, outs))


def validatorapi_submit(impl, share_idx: int, pubshare_of: Mapping[bytes, bytes],
                        submissions: Sequence[Tuple[bytes, bytes, bytes]]) -> None:
    """Component.SubmitAttestations (validatorapi.go:284-306): the local VC's partials
    (pubkey, signing root, signature) verified in one batch; the first failure is returned as
    verifyPartialSig returns it (validatorapi.go:1213-1229)."""
    del share_idx  # the partials carry the node's own share index
    pks, msgs, sigs = [], [], []
    for pubkey, root, sig in submissions:
        if sig == ZERO_SIG:
            raise CallerError("no signature found")
        pks.append(pubshare_of[pubkey])
        msgs.append(root)
        sigs.append(sig)
    for s in impl.verify_batch(pks, msgs, sigs) if pks else []:
        if s != OK:
            raise CallerError(_VERIFY_ERR.get(s, "signature not verified"))


def lock_verify_signatures(impl, public_shares: Sequence[bytes], signature_aggregate: bytes,
                           lock_hash: bytes) -> None:
    """Lock.VerifySignatures' aggregate check (lock.go:165-189): VerifyAggregate over every
    validator's every public share against the lock hash."""
    st = impl.verify_aggregate_batch([list(public_shares)], [signature_aggregate], [lock_hash])[0]
    if st != OK:
        raise _wrap("verify lock signature aggregate", _VERIFY_AGG_ERR.get(st, "signature verification failed"))


def dkg_agg_deposit_data(impl, pubshares_by_dv: Mapping[bytes, Mapping[int, bytes]],
                         partials: Mapping[bytes, Sequence[ParSig]]) -> Dict[bytes, bytes]:
    """aggDepositData (dkg.go:820-899): every partial verified (one batch), every DV's partials
    threshold-aggregated (one batch), every aggregate verified under the DV key (one batch)."""
    keys = list(partials)
    pks, msgs, sigs = [], [], []
    for dv in keys:
        for ps in partials[dv]:
            shares = pubshares_by_dv.get(dv)
            if shares is None:
                raise CallerError("invalid pubkey in deposit data partial signature from peer")
            if ps.share_idx not in shares:
                raise CallerError("invalid pubshare")
            pks.append(shares[ps.share_idx])
            msgs.append(ps.signing_root)
            sigs.append(ps.signature)
    for s in impl.verify_batch(pks, msgs, sigs) if pks else []:
        if s != OK:
            raise CallerError("invalid deposit data partial signature from peer")
    outs, sts = impl.threshold_aggregate_batch([{ps.share_idx: ps.signature for ps in partials[dv]} for dv in keys])
    for s in sts:
        if s != OK:
            raise CallerError(_TA_ERR.get(s, "cannot combine signatures"))
    vst = impl.verify_batch(keys, [partials[dv][0].signing_root for dv in keys], outs)
    for s in vst:
        if s != OK:
            raise _wrap("invalid deposit data aggregated signature", _VERIFY_ERR.get(s, "signature not verified"))
    return dict(zip(keys, outs))


def exit_aggregate(impl, partial_sigs: Sequence[Optional[bytes]]) -> bytes:
    """The exit blob's aggregation (app/obolapi/exit.go:165-194): entry i is share i+1's partial
    signature or None (not pushed yet, ignored)."""
    group = {i + 1: s for i, s in enumerate(partial_sigs) if s}
    outs, sts = impl.threshold_aggregate_batch([group])
    if sts[0] != OK:
        raise _wrap("partial signatures threshold aggregate", _TA_ERR.get(sts[0], "cannot combine signatures"))
    return outs[0]
