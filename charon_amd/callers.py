"""Host-side mirrors of charon's BLS call sites, switched to the batch entry points (SURVEY.md
§8(f)1 and §8(f)4).  Each function keeps the reference's error strings and reports the error the
reference's per-item loop would return first; only the per-item tbls calls are replaced by batch
calls.  INTEGRATION.md §3 gives the same changes as Go patches.

  parsigex_verify_set             core/parsigex/parsigex.go:93-98 + NewEth2Verifier :145-170
                                  (+ eth2util/signing/signing.go:96-115 zero-signature check)
  sigagg_aggregate                core/sigagg/sigagg.go:48-81 + aggregate :83-122 (TA :105, verify :117,
                                  NewVerifier :124-144)
  validatorapi_submit             core/validatorapi/validatorapi.go:284-306 + verifyPartialSig :1213-1229
  lock_verify_signatures          cluster/lock.go:151-197 (VerifyAggregate over every pubshare, :185)
  dkg_agg_deposit_data            dkg/dkg.go:820-899 (n x Verify + ThresholdAggregate + Verify per DV)
  dkg_agg_validator_registrations dkg/dkg.go:901-984 (the same shape over registration roots)
  dkg_agg_lock_hash_sig           dkg/dkg.go:659-703 (Verify of every partial + plain Aggregate)
  dkg_verify_lock_multisig        dkg/dkg.go:595-598 (VerifyAggregate of that aggregate)
  exit_aggregate                  app/obolapi/exit.go:165-194 (ThresholdAggregate of the exit partials)
  exit_aggregate_batch            cmd/exit_fetch.go:120-137 --all: every validator's exit partials in one batch

First-error semantics.  The reference loops check item by item and return at the first failure.
A batch call verifies everything at once, so each mirror (i) runs the cheap per-item pre-checks
(lookups, lengths, zero signature) in loop order up to the first failing one, (ii) batches the
cryptographic checks of every item before it, and (iii) walks the loop order again, returning the
first error of either kind -- exactly the error the reference returns (for the Go map iterations,
exactly the error of that iteration order).

`impl` is any object with the batch methods of charon_amd.tbls.HIPBLS (verify_batch,
threshold_aggregate_batch, aggregate_batch, verify_aggregate_batch).  Messages are the 32-byte
signing roots the callers compute (eth2util/signing.GetDataRoot), or roots computed on the GPU by
charon_amd.signing_roots.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Mapping, Optional, Sequence, Tuple

from .tbls import TblsError, status_error

OK = 0
ZERO_SIG = bytes(96)
_LEN_ERR = "data is not of the correct length"  # tbls/tblsconv/tblsconv.go:46,66


class CallerError(TblsError):
    """The error a reference call site returns (wrapped message, as errors.Wrap prints it)."""


def _wrap(outer: str, inner: str) -> CallerError:
    return CallerError(f"{outer}: {inner}")


def _verr(st: int) -> str:
    return status_error("verify", st)


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
    "invalid partial signature: <NewEth2Verifier error>" (parsigex.go:96, :148-165)."""
    pks, msgs, sigs = [], [], []
    pre: Optional[str] = None
    for pubkey, ps in data_set:
        shares = pubshares_by_key.get(pubkey)
        if shares is None:
            pre = "unknown pubkey, not part of cluster lock"
            break
        pubshare = shares.get(ps.share_idx)
        if pubshare is None:
            pre = "invalid shareIdx"
            break
        if ps.signature == ZERO_SIG:  # signing.go:107-110, before tbls.Verify
            pre = "invalid signature: no signature found"
            break
        pks.append(pubshare)
        msgs.append(ps.signing_root)
        sigs.append(ps.signature)
    if pks and hasattr(impl, "verify_batch_first_error"):
        # the set up to its first failure (hbls_verify_batch_first_error): under attack the library
        # resolves only the first failing item instead of every item's verdict
        first, st = impl.verify_batch_first_error(pks, msgs, sigs)
        if first >= 0:
            raise _wrap("invalid partial signature", "invalid signature: " + _verr(st))
    else:
        for s in impl.verify_batch(pks, msgs, sigs) if pks else []:
            if s != OK:
                raise _wrap("invalid partial signature", "invalid signature: " + _verr(s))
    if pre is not None:
        raise _wrap("invalid partial signature", pre)


def sigagg_aggregate(impl, threshold: int, dv_pubkeys: Mapping[bytes, bytes],
                     sets: Mapping[bytes, Sequence[ParSig]]) -> Dict[bytes, bytes]:
    """Aggregator.Aggregate (sigagg.go:48-81): the validators' partials threshold-aggregated in one
    batch, then every aggregate verified under its DV key in one batch (sigagg.go:117,
    NewVerifier :124-144).  The first validator whose step fails aborts the duty set with
    "threshold aggregate: <error>" (sigagg.go:58)."""
    if not sets:
        raise CallerError("empty partial signed data set")
    keys = list(sets)
    groups: List[Dict[int, bytes]] = []
    pre: Optional[str] = None
    for pk in keys:  # aggregate()'s checks before the TA (sigagg.go:84-101)
        par = sets[pk]
        if len(par) < threshold:
            pre = "require threshold signatures"
            break
        by_idx: Dict[int, bytes] = {}
        for ps in par:
            if len(ps.signature) != 96:
                pre = "signature from core: " + _LEN_ERR
                break
            by_idx[ps.share_idx] = ps.signature
        if pre is not None:
            break
        if len(by_idx) < threshold:
            pre = "number of partial signatures less than threshold"
            break
        groups.append(by_idx)
    done = keys[:len(groups)]
    outs, sts = impl.threshold_aggregate_batch(groups) if groups else ([], [])
    ok = [k for k, s in enumerate(sts) if s == OK]
    vst = dict(zip(ok, impl.verify_batch([dv_pubkeys[done[k]] for k in ok],
                                         [sets[done[k]][0].signing_root for k in ok],
                                         [outs[k] for k in ok]))) if ok else {}
    for k in range(len(done)):
        if sts[k] != OK:
            raise _wrap("threshold aggregate", status_error("threshold_aggregate", sts[k]))
        if vst[k] != OK:
            raise _wrap("threshold aggregate", "aggregate signature verification failed: " + _verr(vst[k]))
    if pre is not None:
        raise _wrap("threshold aggregate", pre)
    return dict(zip(done, outs))


def validatorapi_submit(impl, pubshare_of: Mapping[bytes, bytes],
                        submissions: Sequence[Tuple[bytes, bytes, bytes]]) -> None:
    """Component.SubmitAttestations (validatorapi.go:284-306): the local VC's partials
    (pubkey, signing root, signature) verified in one batch before any set reaches the
    subscribers; the first failing attestation's error is returned as verifyPartialSig returns it
    (validatorapi.go:1213-1229: "unknown public key" from getVerifyShareFunc :121-125, "no signature
    found" from signing.Verify, else the tbls.Verify error)."""
    pks, msgs, sigs = [], [], []
    pre: Optional[str] = None
    for pubkey, root, sig in submissions:
        pubshare = pubshare_of.get(pubkey)
        if pubshare is None:
            pre = "unknown public key"
            break
        if sig == ZERO_SIG:
            pre = "no signature found"
            break
        pks.append(pubshare)
        msgs.append(root)
        sigs.append(sig)
    for s in impl.verify_batch(pks, msgs, sigs) if pks else []:
        if s != OK:
            raise CallerError(_verr(s))
    if pre is not None:
        raise CallerError(pre)


def lock_verify_signatures(impl, public_shares: Sequence[bytes], signature_aggregate: bytes,
                           lock_hash: bytes) -> None:
    """Lock.VerifySignatures' aggregate check (lock.go:165-189): VerifyAggregate over every
    validator's every public share against the lock hash."""
    st = impl.verify_aggregate_batch([list(public_shares)], [signature_aggregate], [lock_hash])[0]
    if st != OK:
        raise _wrap("verify lock signature aggregate", status_error("verify_aggregate", st))


def _dkg_partials(pubshares_by_dv, partials, roots, what: str, missing_msg: Optional[str],
                  sig_ctx: str = "signature from core"):
    """The DKG loops' per-partial pre-checks in loop order (dkg.go:838-869 / :919-950 / :665-682),
    up to the first failure.  Returns (checked items [(dv index, pubshare, root, sig)], complete DVs,
    the first pre-check error or None)."""
    items, complete = [], 0
    for d, dv in enumerate(partials):
        if missing_msg is not None and dv not in roots:
            return items, complete, missing_msg
        for ps in partials[dv]:
            if len(ps.signature) != 96:
                return items, complete, f"{sig_ctx}: {_LEN_ERR}"
            shares = pubshares_by_dv.get(dv)
            if shares is None:
                return items, complete, f"invalid pubkey in {what} partial signature from peer"
            if ps.share_idx not in shares:
                return items, complete, "invalid pubshare"
            items.append((d, shares[ps.share_idx], roots[dv] if roots is not None else ps.signing_root,
                          ps.signature))
        complete = d + 1
    return items, complete, None


def _dkg_threshold_aggregate(impl, pubshares_by_dv, partials, roots, what, missing_msg, agg_err, verify_what=None):
    """aggDepositData / aggValidatorRegistrations (dkg.go:820-899, :901-984) batched: every checked
    partial verified (one batch), every complete DV threshold-aggregated (one batch), every aggregate
    verified under the DV key (one batch); then the first error in the reference's loop order."""
    keys = list(partials)
    items, complete, pre = _dkg_partials(pubshares_by_dv, partials, roots, what, missing_msg)
    vst = impl.verify_batch([p for _, p, _, _ in items], [m for _, _, m, _ in items],
                            [s for _, _, _, s in items]) if items else []
    groups = [{ps.share_idx: ps.signature for ps in partials[keys[d]]} for d in range(complete)]
    outs, tst = impl.threshold_aggregate_batch(groups) if groups else ([], [])
    ok = [d for d in range(complete) if tst[d] == OK]
    ast = dict(zip(ok, impl.verify_batch([keys[d] for d in ok], [roots[keys[d]] for d in ok],
                                         [outs[d] for d in ok]))) if ok else {}
    k = 0
    for d in range(len(keys)):
        while k < len(items) and items[k][0] == d:
            if vst[k] != OK:  # errors.New: the herumi error is not wrapped (dkg.go:866-868)
                raise CallerError(f"invalid {verify_what or what} partial signature from peer")
            k += 1
        if d >= complete:
            break
        if tst[d] != OK:
            raise CallerError(status_error("threshold_aggregate", tst[d]))
        if ast[d] != OK:
            raise _wrap(agg_err, _verr(ast[d]))
    if pre is not None:
        raise CallerError(pre)
    return dict(zip(keys, outs))


def dkg_agg_deposit_data(impl, pubshares_by_dv: Mapping[bytes, Mapping[int, bytes]],
                         partials: Mapping[bytes, Sequence[ParSig]],
                         signing_roots: Mapping[bytes, bytes]) -> Dict[bytes, bytes]:
    """aggDepositData (dkg.go:820-899); signing_roots[dv] = deposit.GetMessageSigningRoot of the
    DV's deposit message (dkg.go:836).  Returns the aggregate signature per DV."""
    return _dkg_threshold_aggregate(impl, pubshares_by_dv, partials, signing_roots, "deposit data",
                                    "deposit message not found", "invalid deposit data aggregated signature")


def dkg_agg_validator_registrations(impl, pubshares_by_dv: Mapping[bytes, Mapping[int, bytes]],
                                    partials: Mapping[bytes, Sequence[ParSig]],
                                    signing_roots: Mapping[bytes, bytes]) -> Dict[bytes, bytes]:
    """aggValidatorRegistrations (dkg.go:901-984); signing_roots[dv] =
    registration.GetMessageSigningRoot of the DV's registration (dkg.go:917).  Returns the
    aggregate signature per DV (setRegistrationSignature's input, dkg.go:974)."""
    # the key lookup says "registrations", the partial check "registration" (dkg.go:938, :956)
    return _dkg_threshold_aggregate(impl, pubshares_by_dv, partials, signing_roots, "validator registrations",
                                    "validator registration not found",
                                    "invalid validator registration aggregated signature", "validator registration")


def dkg_agg_lock_hash_sig(impl, pubshares_by_dv: Mapping[bytes, Mapping[int, bytes]],
                          partials: Mapping[bytes, Sequence[ParSig]], lock_hash: bytes) -> Tuple[bytes, List[bytes]]:
    """aggLockHashSig (dkg.go:659-703): every node's lock-hash partial of every DV verified (one
    batch; the error wraps the tbls error, "invalid lock hash partial signature from peer: ..."),
    then ONE plain BLS aggregate of all of them.  Returns (aggregate, the pubshares in order)."""
    items, _, pre = _dkg_partials(pubshares_by_dv, partials, None, "lock hash", None, "signature from bytes")
    vst = impl.verify_batch([p for _, p, _, _ in items], [lock_hash] * len(items),
                            [s for _, _, _, s in items]) if items else []
    for s in vst:
        if s != OK:
            raise _wrap("invalid lock hash partial signature from peer", _verr(s))
    if pre is not None:
        raise CallerError(pre)
    outs, sts = impl.aggregate_batch([[s for _, _, _, s in items]])
    if sts[0] != OK:
        raise _wrap("bls aggregate Signatures", status_error("aggregate", sts[0]))
    return outs[0], [p for _, p, _, _ in items]


def dkg_verify_lock_multisig(impl, pubkeys: Sequence[bytes], agg_sig: bytes, lock_hash: bytes) -> None:
    """signAndAggLockHash's check of that aggregate (dkg.go:595-598)."""
    st = impl.verify_aggregate_batch([list(pubkeys)], [agg_sig], [lock_hash])[0]
    if st != OK:
        raise _wrap("verify multisignature", status_error("verify_aggregate", st))


def exit_aggregate(impl, partial_sigs: Sequence[Optional[bytes]]) -> bytes:
    """The exit blob's aggregation (app/obolapi/exit.go:165-194): entry i is share i+1's partial
    signature or None (not pushed yet, ignored)."""
    group = {}
    for i, s in enumerate(partial_sigs):
        if not s:
            continue
        if len(s) != 96:
            raise _wrap("invalid partial signature", _LEN_ERR)
        group[i + 1] = s
    outs, sts = impl.threshold_aggregate_batch([group])
    if sts[0] != OK:
        raise _wrap("partial signatures threshold aggregate", status_error("threshold_aggregate", sts[0]))
    return outs[0]


def exit_aggregate_batch(impl, validators: Sequence[Tuple[str, Sequence[Optional[bytes]]]]) -> List[bytes]:
    """`charon exit fetch --all` (cmd/exit_fetch.go:120-137) with INTEGRATION.md's
    AggregateFullExits: every validator's fetched exit partials (entry i = share i+1's signature or
    None) threshold-aggregated in ONE batch; the first validator (in lock order) whose aggregation
    fails aborts with "load full exit data from Obol API: partial signatures threshold aggregate:
    <error>"."""
    groups = []
    pre: Optional[str] = None
    for _, partial_sigs in validators:  # the length pre-check in lock order, up to the first failure
        group = {}
        for i, s in enumerate(partial_sigs):
            if not s:
                continue
            if len(s) != 96:
                pre = _wrap("invalid partial signature", _LEN_ERR).args[0]
                break
            group[i + 1] = s
        if pre is not None:
            break
        groups.append(group)
    outs, sts = impl.threshold_aggregate_batch(groups) if groups else ([], [])
    for st in sts:  # an earlier validator's aggregation error comes first (exit_fetch.go:122-132)
        if st != OK:
            raise _wrap("load full exit data from Obol API",
                        "partial signatures threshold aggregate: " + status_error("threshold_aggregate", st))
    if pre is not None:
        raise _wrap("load full exit data from Obol API", pre)
    return outs
