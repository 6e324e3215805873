"""Diagnosis: device rlc ladders and sums vs the host harness."""
import ctypes
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
dc = ctypes.CDLL(os.path.join(ROOT, "tests", "native", "libhbls_devcheck.so"))
hc = ctypes.CDLL(os.path.join(ROOT, "tests", "native", "libhbls_hostcheck.so"))
k = json.load(open(os.path.join(ROOT, "tests", "golden", "kat_reference.json")))
vs = k["deposit"] * 4
n = len(vs)
pks = b"".join(bytes.fromhex(v["pk"]) for v in vs)
sigs = b"".join(bytes.fromhex(v["sig"]) for v in vs)
rng = random.Random(4)
ab = [rng.getrandbits(32) for _ in range(2 * n)]
ab[0:4] = [1, 0, 0, 1]
abc = (ctypes.c_uint32 * (2 * n))(*ab)
o48, o96, s48, s96 = (ctypes.create_string_buffer(x * n) for x in (48, 96, 48, 96))
print("dc_rlc rc", dc.dc_rlc(pks, sigs, abc, n, o48, o96, s48, s96))
for i in range(n):
    h48, h96 = ctypes.create_string_buffer(48), ctypes.create_string_buffer(96)
    hc.hc_rlc(pks[48 * i:48 * i + 48], sigs[96 * i:96 * i + 96], ab[2 * i], ab[2 * i + 1], h48, h96)
    print(i, "g1", o48.raw[48 * i:48 * i + 48] == h48.raw, "g2", o96.raw[96 * i:96 * i + 96] == h96.raw)
