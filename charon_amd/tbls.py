"""Python mirror of charon's `tbls` package backed by the MI355X library (libhipbls.so).

Reference interface: /root/reference/tbls/tbls.go:27-141 (the 12-method `Implementation`,
`SetImplementation` and the package-level functions) and the semantics and error strings of
/root/reference/tbls/herumi.go.  `HIPBLS` is the drop-in `Implementation`; the batch methods
(`verify_batch`, `threshold_aggregate_batch`, ...) are the new entry points SURVEY.md §8(b)
proposes for sigagg/parsigex (one slot's duties per call).

Types follow tbls.go:16-25: PublicKey = 48 bytes, PrivateKey = 32 bytes, Signature = 96 bytes.
Every hot-path call runs on the GPU; there is no CPU fallback (charon_amd._lib raises
HipBlsUnavailable if the library or device is missing).
"""

from __future__ import annotations

import ctypes
import os
import secrets
import threading
from typing import Dict, Iterable, List, Mapping, Sequence, Tuple

from . import _lib
from ._lib import (BAD_INPUT, BAD_PUBKEY, BAD_SECRET, BAD_SIGNATURE, COMBINE_FAILED, NOT_VERIFIED, OK,
                   check)

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001

PUBKEY_LEN = 48
PRIVKEY_LEN = 32
SIG_LEN = 96


class TblsError(Exception):
    """Raised where the Go implementation returns a non-nil error."""


# herumi.go error strings, by status code and call site.  ONE table: the Python mirror, the caller
# mirrors (callers.py) and the Go shim's switches (INTEGRATION.md verifyStatusErr /
# verifyAggStatusErr / ThresholdAggregateBatch / Aggregate) must all say the same;
# tests/test_go_shim.py parses the Go switches and compares them with this table.
#   kind -> ({status: message}, message of every other non-OK status)
STATUS_ERRORS = {
    "verify": ({
        BAD_PUBKEY: "cannot set compressed public key in Herumi format",   # herumi.go:291
        BAD_SIGNATURE: "cannot unmarshal signature into Herumi signature",  # herumi.go:296
    }, "signature not verified"),                                          # herumi.go:300
    "verify_aggregate": ({
        BAD_PUBKEY: "cannot set compressed public key in Herumi format",   # herumi.go:331
        BAD_SIGNATURE: "cannot unmarshal signature into Herumi signature",  # herumi.go:325
    }, "signature verification failed"),                                   # herumi.go:338
    "threshold_aggregate": ({
        BAD_SIGNATURE: "cannot unmarshal signature into Herumi signature",  # herumi.go:258-262
    }, "cannot combine signatures"),                                       # herumi.go:282
    "aggregate": ({}, "cannot unmarshal signature into Herumi signature"),  # herumi.go:236
}


def status_error(kind: str, st: int):
    """herumi's error message for status `st` of a `kind` call (None for OK)."""
    if st == OK:
        return None
    table, other = STATUS_ERRORS[kind]
    return table.get(st, other)


def _buf(data: bytes):
    return ctypes.create_string_buffer(bytes(data), len(data)) if data else ctypes.create_string_buffer(1)


def _u64_array(vals):
    arr = (ctypes.c_uint64 * max(1, len(vals)))(*vals)
    return arr


def _u32_array(vals):
    return (ctypes.c_uint32 * max(1, len(vals)))(*vals)


def _i64_array(vals):
    return (ctypes.c_int64 * max(1, len(vals)))(*vals)


def _need(b: bytes, n: int, what: str) -> bytes:
    b = bytes(b)
    if len(b) != n:
        raise TblsError(f"invalid {what} length {len(b)}, want {n}")
    return b


def _pack_msgs(msgs: Sequence[bytes]):
    off, lens, blob = [], [], bytearray()
    for m in msgs:
        off.append(len(blob))
        lens.append(len(m))
        blob += m
    return _buf(bytes(blob)), _u64_array(off), _u32_array(lens)


class HIPBLS:
    """tbls.Implementation on the MI355X.  Thread-safe: the library coalesces concurrent
    verification calls into one launch and shards batches over its devices."""

    def __init__(self, device_mask: int = 0):
        self._L = _lib.lib(device_mask)

    # ------------------------------------------------------------------ key management
    def generate_secret_key(self) -> bytes:
        """herumi.go:54-64 (SetByCSPRNG): uniform non-zero scalar < r."""
        while True:
            v = int.from_bytes(secrets.token_bytes(32), "big") & ((1 << 255) - 1)
            if 0 < v < R:
                return v.to_bytes(32, "big")

    def generate_insecure_key(self, random) -> bytes:
        """herumi.go:43-52 + generateInsecureSecret (:346-363): up to 100 reads of 32 bytes."""
        for _ in range(100):
            b = random.read(32)
            if len(b) == 32 and int.from_bytes(b, "big") < R:
                return bytes(b)
        raise TblsError("cannot generate insecure key")

    def secret_to_public_key(self, secret: bytes) -> bytes:
        """herumi.go:66-79."""
        sk = _need(secret, PRIVKEY_LEN, "private key")
        out = ctypes.create_string_buffer(48)
        st = ctypes.create_string_buffer(1)
        check(self._L.hbls_secret_to_public_key_batch(sk, 1, out, st))
        if st.raw[0] != OK:
            if int.from_bytes(sk, "big") >= R:
                raise TblsError("cannot unmarshal secret into Herumi secret key")
            raise TblsError("cannot obtain public key from secret")
        return out.raw

    def _split(self, secret: bytes, total: int, threshold: int, coeffs: List[bytes]) -> Dict[int, bytes]:
        if threshold <= 1:
            raise TblsError("threshold has to be greater than 1")  # herumi.go:140
        sk = _need(secret, PRIVKEY_LEN, "private key")
        if int.from_bytes(sk, "big") >= R:
            raise TblsError("cannot unmarshal bytes into Herumi secret key")
        shares = ctypes.create_string_buffer(32 * max(1, total))
        st = ctypes.create_string_buffer(max(1, total))
        check(self._L.hbls_threshold_split(sk, _buf(b"".join(coeffs)), total, threshold, shares, st))
        if any(st.raw[i] != OK for i in range(total)):
            raise TblsError("cannot set ID on polynomial")
        return {i + 1: shares.raw[32 * i:32 * i + 32] for i in range(total)}

    def threshold_split(self, secret: bytes, total: int, threshold: int) -> Dict[int, bytes]:
        """herumi.go:137-185: random degree-(t-1) polynomial with f(0) = secret, shares f(1..n)."""
        coeffs = [self.generate_secret_key() for _ in range(max(0, threshold - 1))]
        return self._split(secret, total, threshold, coeffs)

    def threshold_split_insecure(self, secret: bytes, total: int, threshold: int, random) -> Dict[int, bytes]:
        """herumi.go:83-135 (coefficients from the caller's reader)."""
        if threshold <= 1:
            raise TblsError("threshold has to be greater than 1")
        coeffs = [self.generate_insecure_key(random) for _ in range(threshold - 1)]
        return self._split(secret, total, threshold, coeffs)

    def recover_secret(self, shares: Mapping[int, bytes], total: int = 0, threshold: int = 0) -> bytes:
        """herumi.go:187-223: Lagrange interpolation at 0 over Fr."""
        ids = list(shares.keys())
        blob = b"".join(_need(shares[i], PRIVKEY_LEN, "private key") for i in ids)
        out = ctypes.create_string_buffer(32)
        st = ctypes.create_string_buffer(1)
        check(self._L.hbls_recover_secret(_buf(blob), _i64_array(ids), len(ids), out, st))
        if st.raw[0] == BAD_SECRET:
            raise TblsError("cannot unmarshal key with into Herumi secret key")
        if st.raw[0] != OK:
            raise TblsError("cannot recover full private key from partial keys")
        return out.raw

    def cache_pubkeys(self, pks: Sequence[bytes]) -> int:
        """Add public keys to the library's key cache (hbls_pubkey_cache_add): later verifications
        take them decompressed and subgroup-checked from it.  charon would add its cluster lock's
        pubshares at startup.  Returns the number of cached keys."""
        blob = b"".join(_need(p, PUBKEY_LEN, "public key") for p in pks)
        if blob:
            check(self._L.hbls_pubkey_cache_add(_buf(blob), len(pks)))
        return int(self._L.hbls_pubkey_cache_size())

    def clear_pubkey_cache(self) -> None:
        check(self._L.hbls_pubkey_cache_clear())

    # ------------------------------------------------------------------ signatures
    def sign(self, private_key: bytes, data: bytes) -> bytes:
        """herumi.go:306-316."""
        return self.sign_batch([private_key], [data])[0]

    def sign_batch(self, sks: Sequence[bytes], msgs: Sequence[bytes]) -> List[bytes]:
        n = len(sks)
        if n != len(msgs):
            raise TblsError("sign_batch: length mismatch")
        if n == 0:
            return []
        blob = b"".join(_need(s, PRIVKEY_LEN, "private key") for s in sks)
        mb, mo, ml = _pack_msgs([bytes(m) for m in msgs])
        out = ctypes.create_string_buffer(96 * n)
        st = ctypes.create_string_buffer(n)
        check(self._L.hbls_sign_batch(_buf(blob), mb, mo, ml, n, out, st))
        res = []
        for i in range(n):
            if st.raw[i] != OK:
                raise TblsError("cannot unmarshal secret into Herumi secret key")
            res.append(out.raw[96 * i:96 * i + 96])
        return res

    def verify(self, compressed_public_key: bytes, data: bytes, signature: bytes) -> None:
        """herumi.go:288-304; raises TblsError with herumi's message, returns None on success."""
        st = self.verify_batch([compressed_public_key], [data], [signature])[0]
        if st != OK:
            raise TblsError(status_error("verify", st))

    def verify_batch(self, pks: Sequence[bytes], msgs: Sequence[bytes], sigs: Sequence[bytes]) -> List[int]:
        """Batch tbls.Verify: one status code per item (0 = verified)."""
        n = len(pks)
        if not (n == len(msgs) == len(sigs)):
            raise TblsError("verify_batch: length mismatch")
        if n == 0:
            return []
        pk_blob = b"".join(_need(p, PUBKEY_LEN, "public key") for p in pks)
        sig_blob = b"".join(_need(s, SIG_LEN, "signature") for s in sigs)
        mb, mo, ml = _pack_msgs([bytes(m) for m in msgs])
        st = ctypes.create_string_buffer(n)
        check(self._L.hbls_verify_batch(_buf(pk_blob), _buf(sig_blob), mb, mo, ml, n, st))
        return list(st.raw[:n])

    def verify_batch_first_error(self, pks: Sequence[bytes], msgs: Sequence[bytes],
                                 sigs: Sequence[bytes]) -> Tuple[int, int]:
        """Batch tbls.Verify of an ordered set up to its first failure (hbls_verify_batch_first_error):
        (index of the first failing item, its status), or (-1, OK) when every item verifies -- the
        loops of parsigex.go:93-98 / sigagg.go:56-63 that return the first error."""
        n = len(pks)
        if not (n == len(msgs) == len(sigs)):
            raise TblsError("verify_batch_first_error: length mismatch")
        if n == 0:
            return -1, OK
        pk_blob = b"".join(_need(p, PUBKEY_LEN, "public key") for p in pks)
        sig_blob = b"".join(_need(s, SIG_LEN, "signature") for s in sigs)
        mb, mo, ml = _pack_msgs([bytes(m) for m in msgs])
        first = ctypes.c_int64(-1)
        fst = ctypes.c_uint8(0)
        check(self._L.hbls_verify_batch_first_error(_buf(pk_blob), _buf(sig_blob), mb, mo, ml, n, ctypes.byref(first),
                                                    ctypes.byref(fst), None))
        return int(first.value), int(fst.value) if first.value >= 0 else OK

    def threshold_aggregate(self, partial_signatures_by_index: Mapping[int, bytes]) -> bytes:
        """herumi.go:249-286."""
        outs, sts = self.threshold_aggregate_batch([partial_signatures_by_index])
        if sts[0] != OK:
            raise TblsError(status_error("threshold_aggregate", sts[0]))
        return outs[0]

    def threshold_aggregate_batch(self, groups: Sequence[Mapping[int, bytes]]) -> Tuple[List[bytes], List[int]]:
        """Batch tbls.ThresholdAggregate: one (signature, status) per group."""
        g = len(groups)
        if g == 0:
            return [], []
        sig_blob, idx, off = bytearray(), [], [0]
        for grp in groups:
            for k, s in grp.items():
                sig_blob += _need(s, SIG_LEN, "signature")
                idx.append(int(k))
            off.append(len(idx))
        out = ctypes.create_string_buffer(96 * g)
        st = ctypes.create_string_buffer(g)
        check(self._L.hbls_threshold_aggregate_batch(_buf(bytes(sig_blob)), _i64_array(idx), _u32_array(off), g, out,
                                                     st))
        return [out.raw[96 * i:96 * i + 96] for i in range(g)], list(st.raw[:g])

    def aggregate(self, signs: Sequence[bytes]) -> bytes:
        """herumi.go:225-247 (empty input -> infinity encoding)."""
        outs, sts = self.aggregate_batch([signs])
        if sts[0] != OK:
            raise TblsError(status_error("aggregate", sts[0]))
        return outs[0]

    def aggregate_batch(self, groups: Sequence[Sequence[bytes]]) -> Tuple[List[bytes], List[int]]:
        g = len(groups)
        if g == 0:
            return [], []
        sig_blob, off = bytearray(), [0]
        for grp in groups:
            for s in grp:
                sig_blob += _need(s, SIG_LEN, "signature")
            off.append(off[-1] + len(grp))
        out = ctypes.create_string_buffer(96 * g)
        st = ctypes.create_string_buffer(g)
        check(self._L.hbls_aggregate_batch(_buf(bytes(sig_blob)), _u32_array(off), g, out, st))
        return [out.raw[96 * i:96 * i + 96] for i in range(g)], list(st.raw[:g])

    def verify_aggregate(self, public_shares: Sequence[bytes], signature: bytes, data: bytes) -> None:
        """herumi.go:318-342 (FastAggregateVerify)."""
        st = self.verify_aggregate_batch([public_shares], [signature], [data])[0]
        if st != OK:
            raise TblsError(status_error("verify_aggregate", st))

    def verify_aggregate_batch(self, pk_groups: Sequence[Sequence[bytes]], sigs: Sequence[bytes],
                               msgs: Sequence[bytes]) -> List[int]:
        g = len(pk_groups)
        if not (g == len(sigs) == len(msgs)):
            raise TblsError("verify_aggregate_batch: length mismatch")
        if g == 0:
            return []
        pk_blob, off = bytearray(), [0]
        for grp in pk_groups:
            for p in grp:
                pk_blob += _need(p, PUBKEY_LEN, "public key")
            off.append(off[-1] + len(grp))
        sig_blob = b"".join(_need(s, SIG_LEN, "signature") for s in sigs)
        mb, mo, ml = _pack_msgs([bytes(m) for m in msgs])
        st = ctypes.create_string_buffer(g)
        check(self._L.hbls_verify_aggregate_batch(_buf(bytes(pk_blob)), _u32_array(off), _buf(sig_blob), mb, mo, ml,
                                                  g, st))
        return list(st.raw[:g])


# ---------------------------------------------------------------------- package level API
# tbls.go:11-14, 71-141: a swappable implementation behind package-level functions.
_impl = None
_impl_lock = threading.Lock()


def set_implementation(new_impl) -> None:
    global _impl
    with _impl_lock:
        _impl = new_impl


def _get():
    global _impl
    if _impl is None:
        with _impl_lock:
            if _impl is None:
                _impl = HIPBLS()
    return _impl


def generate_secret_key() -> bytes:
    return _get().generate_secret_key()


def generate_insecure_key(random) -> bytes:
    return _get().generate_insecure_key(random)


def secret_to_public_key(secret: bytes) -> bytes:
    return _get().secret_to_public_key(secret)


def threshold_split(secret: bytes, total: int, threshold: int) -> Dict[int, bytes]:
    return _get().threshold_split(secret, total, threshold)


def threshold_split_insecure(secret: bytes, total: int, threshold: int, random) -> Dict[int, bytes]:
    return _get().threshold_split_insecure(secret, total, threshold, random)


def recover_secret(shares: Mapping[int, bytes], total: int, threshold: int) -> bytes:
    return _get().recover_secret(shares, total, threshold)


def threshold_aggregate(partial_signatures_by_index: Mapping[int, bytes]) -> bytes:
    return _get().threshold_aggregate(partial_signatures_by_index)


def verify(compressed_public_key: bytes, data: bytes, signature: bytes) -> None:
    return _get().verify(compressed_public_key, data, signature)


def sign(private_key: bytes, data: bytes) -> bytes:
    return _get().sign(private_key, data)


def verify_aggregate(shares: Sequence[bytes], signature: bytes, data: bytes) -> None:
    return _get().verify_aggregate(shares, signature, data)


def aggregate(signs: Sequence[bytes]) -> bytes:
    return _get().aggregate(signs)
