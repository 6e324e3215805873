"""Diagnosis: vbatch.hip k_rlc outputs vs the host harness."""
import ctypes
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
dc = ctypes.CDLL(os.path.join(ROOT, "tests", "native", "libhbls_devcheck_vb.so"))
hc = ctypes.CDLL(os.path.join(ROOT, "tests", "native", "libhbls_hostcheck.so"))
k = json.load(open(os.path.join(ROOT, "tests", "golden", "kat_reference.json")))
vs = k["deposit"]
n = len(vs)
pks = b"".join(bytes.fromhex(v["pk"]) for v in vs)
sigs = b"".join(bytes.fromhex(v["sig"]) for v in vs)
key = (ctypes.c_uint32 * 8)(*range(1, 9))
goff = (ctypes.c_uint32 * 2)(0, n)
G1J, G2J = 36 * 4 if False else 0, 0
import sys
g1b = int(sys.argv[1]) if len(sys.argv) > 1 else 144
g2b = int(sys.argv[2]) if len(sys.argv) > 2 else 288
pr = ctypes.create_string_buffer(g1b * n)
sr = ctypes.create_string_buffer(g2b * n)
gp = ctypes.create_string_buffer(160)
gst = ctypes.create_string_buffer(1)
print("rc", dc.dc_vb_rlc(pks, sigs, n, goff, 1, key, pr, sr, gp, gst))
abl = []
for i in range(n):
    ab = (ctypes.c_uint32 * 2)()
    hc.hc_rlc_coeffs(key, i, ab)
    abl += list(ab)
h = ctypes.create_string_buffer(48)
hc.hc_rlc_sum_g1(n, pks, (ctypes.c_uint32 * (2 * n))(*abl), h)
d = ctypes.create_string_buffer(48)
hc.hc_g1a_compress(gp.raw, d)
print("gst", gst.raw[0], "group P equal", d.raw == h.raw, d.raw.hex()[:32], h.raw.hex()[:32])
for i in range(n):
    ab = (ctypes.c_uint32 * 2)()
    hc.hc_rlc_coeffs(key, i, ab)
    h48, h96 = ctypes.create_string_buffer(48), ctypes.create_string_buffer(96)
    hc.hc_rlc(pks[48 * i:48 * i + 48], sigs[96 * i:96 * i + 96], ab[0], ab[1], h48, h96)
    d48, d96 = ctypes.create_string_buffer(48), ctypes.create_string_buffer(96)
    hc.hc_jac_compress(pr.raw[g1b * i:g1b * (i + 1)], d48, sr.raw[g2b * i:g2b * (i + 1)], d96)
    print(i, list(ab), "g1", d48.raw == h48.raw, "g2", d96.raw == h96.raw, pr.raw[g1b * i:g1b * i + 16].hex())
# sums of the raw device points: device loop / device straight-line / host
o, ob, h = ctypes.create_string_buffer(48), ctypes.create_string_buffer(48), ctypes.create_string_buffer(48)
print("dc_sum rc", dc.dc_sum(pr.raw, n, o, ob))
hc.hc_sum_raw(pr.raw, n, h)
h2 = ctypes.create_string_buffer(48)
hc.hc_sum_raw(pr.raw, 2, h2)
print("loop sum == host", o.raw == h.raw, " 2-sum == host", ob.raw == h2.raw, " host sum == group P (host rlc)",
      h.raw == hcsum.raw if False else None)
open(os.path.join(ROOT, "gpurun_out", "probe_vb_pr.bin"), "wb").write(pr.raw)
open(os.path.join(ROOT, "gpurun_out", "probe_vb_gp.bin"), "wb").write(gp.raw)
