"""Diagnosis: which verification groups pass their combined check (HBLS_STATS counters)."""
import ctypes
import hashlib
import os
import sys

os.environ["HBLS_STATS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from charon_amd import _lib, tbls  # noqa: E402

impl = tbls.HIPBLS()
L = _lib.load_library()


def stats():
    out = (ctypes.c_uint64 * 3)()
    L.hbls_stats(out, 3)
    return list(out)


def run(name, pks, msgs, sigs):
    s0 = stats()
    st = impl.verify_batch(pks, msgs, sigs)
    s1 = stats()
    print(f"{name:40s} statuses {st[:12]} items/groups/fallback {[b - a for a, b in zip(s0, s1)]}", flush=True)


keys = [impl.generate_secret_key() for _ in range(8)]
m = hashlib.sha256(b"probe").digest()
sigs = impl.sign_batch(keys, [m] * 8)
pks = [impl.secret_to_public_key(k) for k in keys]
run("one item", pks[:1], [m], sigs[:1])
run("group of 2", pks[:2], [m] * 2, sigs[:2])
run("group of 8", pks, [m] * 8, sigs)
ms = [hashlib.sha256(b"probe %d" % i).digest() for i in range(8)]
sigs2 = impl.sign_batch(keys, ms)
run("8 singletons", pks, ms, sigs2)
