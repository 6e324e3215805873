"""Diagnosis: device jac_add (general Z) vs the host harness, fast and standard translation units."""
import ctypes
import json
import os
import random

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
hc = ctypes.CDLL(os.path.join(ROOT, "tests", "native", "libhbls_hostcheck.so"))
k = json.load(open(os.path.join(ROOT, "tests", "golden", "kat_reference.json")))
vs = k["deposit"] * 4
n = len(vs)
pks = b"".join(bytes.fromhex(v["pk"]) for v in vs)
sigs = b"".join(bytes.fromhex(v["sig"]) for v in vs)
rng = random.Random(8)
ks = [rng.getrandbits(32) | 1 for _ in range(2 * n)]
kc = (ctypes.c_uint32 * (2 * n))(*ks)
for lib in ("libhbls_devcheck_fast.so", "libhbls_devcheck_std.so"):
    dc = ctypes.CDLL(os.path.join(ROOT, "tests", "native", lib))
    o48, o96 = ctypes.create_string_buffer(48 * n), ctypes.create_string_buffer(96 * n)
    rc = dc.dc_jac_add(pks, sigs, kc, n, o48, o96)
    g1ok = g2ok = 0
    for i in range(n):
        h48, h96 = ctypes.create_string_buffer(48), ctypes.create_string_buffer(96)
        hc.hc_jac_add(pks[48 * i:48 * i + 48], sigs[96 * i:96 * i + 96], ks[2 * i], ks[2 * i + 1], h48, h96)
        g1ok += o48.raw[48 * i:48 * i + 48] == h48.raw
        g2ok += o96.raw[96 * i:96 * i + 96] == h96.raw
    print(lib, "rc", rc, "g1 ok", g1ok, "/", n, "g2 ok", g2ok, "/", n, flush=True)
