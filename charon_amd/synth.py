"""Deterministic synthetic clusters for the benchmark and the scale tests.

A cluster of V validators with n operators and threshold t, derived from a seed with SHA-256 so
that every run (and every rank) regenerates identical inputs:

    root secret   s_v     = SHA256("sk"   || seed || v)      mod r   (non-zero)
    coefficients  a_{v,k} = SHA256("poly" || seed || v || k) mod r,  k = 1 .. t-1
    shares        s_{v,i} = f_v(i) = s_v + sum_k a_{v,k} i^k,  i = 1 .. n   (1-based share indices,
                            /root/reference/app/app.go:391-392, cluster/test_cluster.go:57)
    messages      shared:   m_j = SHA256("msg" || seed || j), validator v signs m_{v mod M}
                            (one AttestationData root per committee)
                  distinct: m_v = SHA256("msg" || seed || v)  (C3)

v, k, j are encoded as 8-byte little-endian integers.  Only host-side bookkeeping lives here;
public keys and signatures are produced by the GPU library (hbls_secret_to_public_key_batch,
hbls_sign_batch) and checked against the KAT-pinned arithmetic by tests/.
"""

from __future__ import annotations

import hashlib
import struct
from dataclasses import dataclass
from typing import List

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
DEFAULT_SEED = 0x5EEDC4A7


def _h(tag: bytes, seed: int, *ints: int) -> int:
    m = hashlib.sha256(tag)
    m.update(struct.pack("<Q", seed))
    for x in ints:
        m.update(struct.pack("<Q", x))
    return int.from_bytes(m.digest(), "big")


@dataclass
class Cluster:
    n_validators: int
    n: int
    t: int
    root_sks: List[bytes]          # V x 32 B
    share_sks: List[bytes]         # V*n x 32 B, validator-major, share i at [v*n + i-1]
    msgs: List[bytes]              # distinct messages
    msg_of_validator: List[int]    # V indices into msgs


def make_cluster(n_validators: int, n: int, t: int, *, seed: int = DEFAULT_SEED, first_validator: int = 0,
                 n_msgs: int = 64, distinct_messages: bool = False) -> Cluster:
    if not (1 <= t <= n):
        raise ValueError("need 1 <= t <= n")
    root, shares = [], []
    for v in range(first_validator, first_validator + n_validators):
        s = _h(b"sk", seed, v) % R or 1
        coeffs = [_h(b"poly", seed, v, k) % R for k in range(1, t)]
        root.append(s.to_bytes(32, "big"))
        for i in range(1, n + 1):
            acc = 0
            for c in reversed(coeffs):
                acc = (acc + c) * i % R
            shares.append(((acc + s) % R).to_bytes(32, "big"))
    if distinct_messages:
        msgs = [_h(b"msg", seed, v).to_bytes(32, "big") for v in range(first_validator, first_validator + n_validators)]
        which = list(range(n_validators))
    else:
        msgs = [_h(b"msg", seed, j).to_bytes(32, "big") for j in range(n_msgs)]
        which = [(first_validator + v) % n_msgs for v in range(n_validators)]
    return Cluster(n_validators, n, t, root, shares, msgs, which)
