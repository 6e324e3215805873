#!/usr/bin/env python3
"""GPU diagnosis: single-item host-buffer Verify calls on an idle library -- wall time per call and,
with HBLS_HOST_TIMING=1 (stderr), the host phases.  Usage: diag_single.py [calls]"""
import hashlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from charon_amd import tbls  # noqa: E402

impl = tbls.HIPBLS()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
sk = impl.generate_secret_key()
pk = impl.secret_to_public_key(sk)
msgs = [hashlib.sha256(b"single %d" % k).digest() for k in range(n + 2)]
sigs = impl.sign_batch([sk] * len(msgs), msgs)
impl.verify_batch([pk], [msgs[0]], [sigs[0]])  # warm
impl.verify_batch([pk], [msgs[1]], [sigs[1]])
lat = []
for k in range(2, n + 2):
    t0 = time.perf_counter()
    st = impl.verify_batch([pk], [msgs[k]], [sigs[k]])
    lat.append((time.perf_counter() - t0) * 1e3)
    assert st == [0]
print("single-call latency ms:", [round(x, 2) for x in lat], "median", round(sorted(lat)[len(lat) // 2], 2))
