"""Signing roots on the GPU: the 32-byte messages charon verifies, built from
the duty data instead of on the host.

    GetDataRoot(domain, object_root) = SSZ SigningData{object_root, domain}.HashTreeRoot
                                      (eth2util/signing/signing.go:63-77)
    attestation object root          = phase0.AttestationData.HashTreeRoot
                                      (core/signeddata.go Attestation.MessageRoot)

`attestation_signing_roots` takes AttestationData in its 128-byte SSZ encoding (what charon
receives on the wire and marshals with go-eth2-client); `signing_roots` takes object roots the
caller computed for other duty types.  Domains come from signing.GetDomain (fork schedule and
genesis validators root), one per item or one shared.  Both run as HIP kernels
(charon_amd/csrc/roots.hip) through the C ABI; there is no CPU path.
"""

from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from .tbls import TblsError

ATTESTATION_DATA_LEN = 128


def _p(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data)


def _domains(domains: Sequence[bytes], dom_idx: Optional[Sequence[int]], n: int):
    if not domains or any(len(d) != 32 for d in domains):
        raise TblsError("signing roots: domains must be 32 bytes each")
    dom = np.frombuffer(b"".join(domains), dtype=np.uint8).copy()
    idx = None
    if dom_idx is not None:
        if len(dom_idx) != n:
            raise TblsError("signing roots: one domain index per item")
        idx = np.asarray(dom_idx, dtype=np.uint32)
    return dom, idx


def _run(fn_name: str, data: np.ndarray, n: int, domains, dom_idx) -> List[bytes]:
    dom, idx = _domains(domains, dom_idx, n)
    out = np.zeros(32 * max(n, 1), dtype=np.uint8)
    if n:
        L = _lib.lib()
        rc = getattr(L, fn_name)(_p(data), n, _p(dom), len(domains), None if idx is None else _p(idx), _p(out))
        if rc != 0:
            raise TblsError(L.hbls_last_error().decode(errors="replace"))
    return [out[32 * i:32 * i + 32].tobytes() for i in range(n)]


def attestation_signing_roots(data: Sequence[bytes], domains: Sequence[bytes],
                              dom_idx: Optional[Sequence[int]] = None) -> List[bytes]:
    """Signing roots of SSZ-encoded AttestationData (128 bytes each)."""
    if any(len(d) != ATTESTATION_DATA_LEN for d in data):
        raise TblsError("signing roots: AttestationData must be 128 SSZ bytes")
    blob = np.frombuffer(b"".join(data) or b"\0", dtype=np.uint8).copy()
    return _run("hbls_attestation_signing_roots", blob, len(data), domains, dom_idx)


def signing_roots(object_roots: Sequence[bytes], domains: Sequence[bytes],
                  dom_idx: Optional[Sequence[int]] = None) -> List[bytes]:
    """GetDataRoot of caller-computed object roots (32 bytes each)."""
    if any(len(r) != 32 for r in object_roots):
        raise TblsError("signing roots: object roots must be 32 bytes")
    blob = np.frombuffer(b"".join(object_roots) or b"\0", dtype=np.uint8).copy()
    return _run("hbls_signing_roots", blob, len(object_roots), domains, dom_idx)


# hbls_duty_signing_roots kinds (include/hipbls.h): the other duty types of core/signeddata.go
AGGREGATE_AND_PROOF = 1        # SignedAggregateAndProof: phase0.AggregateAndProof SSZ
CONTRIBUTION_AND_PROOF = 2     # SignedSyncContributionAndProof: altair.ContributionAndProof SSZ (264 B)
SYNC_SELECTION = 3             # SyncContributionAndProof / SyncCommitteeSelection: slot || subcommittee_index
SLOT = 4                       # BeaconCommitteeSelection: the uint64 slot (8 B little-endian)
SYNC_MESSAGE = 5               # SignedSyncMessage: the beacon block root (32 B)
VALIDATOR_REGISTRATION = 6     # VersionedSignedValidatorRegistration: v1.ValidatorRegistration SSZ (84 B)
VOLUNTARY_EXIT = 7             # SignedVoluntaryExit: phase0.VoluntaryExit SSZ (16 B)
RANDAO = 8                     # SignedRandao: the uint64 epoch (8 B little-endian)
BLOCK_HEADER = 9               # VersionedSignedProposal: phase0.BeaconBlockHeader SSZ (112 B, body root given)


def duty_signing_roots(kind: int, objects: Sequence[bytes], domains: Sequence[bytes],
                       dom_idx: Optional[Sequence[int]] = None):
    """Signing roots of SSZ-encoded duty objects of one kind (the object root computed on the
    device, core/signeddata.go MessageRoot).  Returns (roots, statuses): status 6 (HBLS_BAD_INPUT)
    for a malformed object, whose root is then all zero."""
    n = len(objects)
    dom, idx = _domains(domains, dom_idx, n)
    blob = np.frombuffer(b"".join(objects) or b"\0", dtype=np.uint8).copy()
    lens = np.asarray([len(o) for o in objects] or [0], dtype=np.uint32)
    offs = np.zeros(max(n, 1), dtype=np.uint64)
    if n:
        offs[1:n] = np.cumsum(lens[:-1], dtype=np.uint64)
    out = np.zeros(32 * max(n, 1), dtype=np.uint8)
    st = np.zeros(max(n, 1), dtype=np.uint8)
    if n:
        L = _lib.lib()
        rc = L.hbls_duty_signing_roots(kind, _p(blob), _p(offs), _p(lens), n, _p(dom), len(domains),
                                       None if idx is None else _p(idx), _p(out), _p(st))
        if rc != 0:
            raise TblsError(L.hbls_last_error().decode(errors="replace"))
    return [out[32 * i:32 * i + 32].tobytes() for i in range(n)], [int(x) for x in st[:n]]
