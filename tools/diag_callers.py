#!/usr/bin/env python3
"""GPU diagnosis of the coalesced single-item path: `threads` host threads calling
hbls_verify_batch with one item each for `seconds`, the library's per-batch host timing
(HBLS_HOST_TIMING=1, stderr) summarised: batch sizes, lock wait, enqueue and device time.
Usage: diag_callers.py [threads] [seconds]   (run with HBLS_HOST_TIMING=1 2> file)"""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import bench  # noqa: E402
from charon_amd import _lib  # noqa: E402

threads = int(sys.argv[1]) if len(sys.argv) > 1 else 64
seconds = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
L = _lib.load_library()
wl = bench.WORKLOADS["c2"]
d = bench.setup_inputs(L, wl, wl["validators"], 0)
NP = d["NP"]
pks, sigs, msgs = d["pks"], d["sigs"], d["item_msgs"]
off0 = np.zeros(1, dtype=np.uint64)
len32 = np.full(1, 32, dtype=np.uint32)
stop = time.perf_counter() + seconds
counts = [0] * threads


def worker(w):
    st = np.zeros(1, dtype=np.uint8)
    k = w
    while time.perf_counter() < stop:
        i = (k * 104729) % NP
        L.hbls_verify_batch(bench._p(pks[48 * i:]), bench._p(sigs[96 * i:]), bench._p(msgs[32 * i:]), bench._p(off0),
                            bench._p(len32), 1, bench._p(st))
        counts[w] += 1
        k += threads


if len(sys.argv) > 3 and sys.argv[3] == "batch":  # one caller, `threads` items per call (a trace target)
    m = threads
    st = np.zeros(m, dtype=np.uint8)
    idx = [(k * 104729) % NP for k in range(m)]
    P = np.concatenate([pks[48 * i:48 * i + 48] for i in idx])
    S = np.concatenate([sigs[96 * i:96 * i + 96] for i in idx])
    M = np.concatenate([msgs[32 * i:32 * i + 32] for i in idx])
    off = np.arange(m, dtype=np.uint64) * 32
    ln = np.full(m, 32, dtype=np.uint32)
    ts = []
    for _ in range(12):
        t1 = time.perf_counter()
        L.hbls_verify_batch(bench._p(P), bench._p(S), bench._p(M), bench._p(off), bench._p(ln), m, bench._p(st))
        ts.append((time.perf_counter() - t1) * 1e3)
    print(f"batch of {m}: ms", [round(x, 2) for x in ts], "all ok", not st.any(), flush=True)
    sys.exit(0)
t0 = time.perf_counter()
ths = [threading.Thread(target=worker, args=(w,)) for w in range(threads)]
for th in ths:
    th.start()
for th in ths:
    th.join()
print(f"{threads} threads: {sum(counts) / (time.perf_counter() - t0):.0f} calls/s", flush=True)
