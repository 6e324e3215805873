"""The host-buffer Verify's message dedup (charon_amd/csrc/msgtable.h): the parallel version of
large calls partitions the items into the same classes of equal messages as the sequential one,
every id naming its items' bytes -- messages of several lengths (0, 32, 33, 100 bytes), many and
few duplicates."""
import ctypes
import random

import numpy as np
import pytest


@pytest.fixture(scope="module")
def hc():
    from charon_amd.build import build_hostcheck
    lib = ctypes.CDLL(build_hostcheck(verbose=False))
    lib.hc_dedup.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    lib.hc_dedup.restype = ctypes.c_long
    return lib


def _items(rng, n, distinct):
    pool = [rng.randbytes(rng.choice((0, 32, 32, 32, 33, 100))) for _ in range(distinct)]
    msgs = [pool[rng.randrange(distinct)] for _ in range(n)]
    blob = b"".join(msgs) or b"\0"
    off = np.zeros(n, dtype=np.uint64)
    off[1:] = np.cumsum([len(m) for m in msgs[:-1]], dtype=np.uint64)
    ln = np.array([len(m) for m in msgs], dtype=np.uint32)
    return msgs, np.frombuffer(blob, dtype=np.uint8).copy(), off, ln


@pytest.mark.parametrize("n,distinct", [(1000, 3), (70000, 7000), (200000, 200000)])
def test_parallel_dedup_same_classes(hc, n, distinct):
    rng = random.Random(n + distinct)
    msgs, blob, off, ln = _items(rng, n, distinct)
    want = {}
    classes = [want.setdefault(m, len(want)) for m in msgs]
    for threads in (0, 4, 8):
        idx = np.zeros(n, dtype=np.uint32)
        got = hc.hc_dedup(blob.ctypes.data, off.ctypes.data, ln.ctypes.data, n, threads, idx.ctypes.data)
        assert got == len(want), threads
        # same partition: a bijection between the ids and the true classes
        pairs = set(zip(classes, idx.tolist()))
        assert len(pairs) == len(want), threads
