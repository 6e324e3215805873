"""Child process of tests/test_gpu_knobs.py: the library initialised with every environment
setting it reads at hbls_init at a NON-default value (the parent passes them), then a small
workload through the host-buffer entry points -- Verify with bad items, concurrent single-item
callers (the coalescer), ThresholdAggregate (the signature cache), first-error Verify -- checked
against the construction.  Prints one JSON line of results."""
import ctypes
import json
import os
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401  (the HIP runtime first: charon_amd/_lib.py)

import bench  # noqa: E402
from charon_amd import _lib  # noqa: E402


def _p(x):
    return ctypes.c_void_p(x.ctypes.data)


def main():
    L = _lib.lib()
    wl = dict(validators=600, n=4, t=3, distinct=False, n_msgs=8)
    d = bench.setup_inputs(L, wl, wl["validators"], 0)
    NP, V = d["NP"], d["V"]
    sigs = d["sigs"].reshape(NP, 96).copy()
    bad = [7, 1000, NP - 2]
    for i in bad:
        sigs[i] = sigs[(i + 1) % NP]
    sigs = sigs.reshape(-1).copy()
    st = np.full(NP, 255, dtype=np.uint8)
    rc = L.hbls_verify_batch(_p(d["pks"]), _p(sigs), _p(d["item_msgs"]), _p(d["item_off"]), _p(d["item_len"]), NP,
                             _p(st))
    want = np.zeros(NP, dtype=np.uint8)
    want[bad] = 3
    res = {"verify_ok": rc == 0 and bool(np.array_equal(st, want))}
    first = ctypes.c_int64(-2)
    fst = ctypes.c_uint8(0)
    rc = L.hbls_verify_batch_first_error(_p(d["pks"]), _p(sigs), _p(d["item_msgs"]), _p(d["item_off"]),
                                         _p(d["item_len"]), NP, ctypes.byref(first), ctypes.byref(fst), None)
    res["first_error_ok"] = rc == 0 and first.value == bad[0] and fst.value == 3
    out = np.zeros(V * 96, dtype=np.uint8)
    tst = np.zeros(V, dtype=np.uint8)
    rc = L.hbls_threshold_aggregate_batch(_p(d["ta_sigs"]), _p(d["ta_idx"]), _p(d["grp_off"]), V, _p(out), _p(tst))
    res["aggregate_ok"] = rc == 0 and not tst.any() and bool(np.array_equal(out, d["root_sigs"]))
    if not res["aggregate_ok"]:
        res["aggregate_detail"] = {"rc": int(rc), "bad_status": int((tst != 0).sum()),
                                   "statuses": sorted(set(int(x) for x in tst)),
                                   "wrong": int((out.reshape(V, 96) != d["root_sigs"].reshape(V, 96)).any(axis=1).sum()),
                                   "first_wrong": [int(x) for x in np.nonzero(
                                       (out.reshape(V, 96) != d["root_sigs"].reshape(V, 96)).any(axis=1))[0][:8]]}
    # back to back on the same host-call contexts: a Verify whose signature-cache put (after the
    # call returned) still reads its staging buffers, then an aggregation that uploads into them
    ok = True
    for _ in range(10):
        rc1 = L.hbls_verify_batch_first_error(_p(d["pks"]), _p(sigs), _p(d["item_msgs"]), _p(d["item_off"]),
                                              _p(d["item_len"]), NP, ctypes.byref(first), ctypes.byref(fst), None)
        rc2 = L.hbls_threshold_aggregate_batch(_p(d["ta_sigs"]), _p(d["ta_idx"]), _p(d["grp_off"]), V, _p(out),
                                               _p(tst))
        ok = ok and rc1 == 0 and rc2 == 0 and first.value == bad[0] and not tst.any() and \
            bool(np.array_equal(out, d["root_sigs"]))
    res["back_to_back_ok"] = ok
    errs = []
    off0 = np.zeros(1, dtype=np.uint64)
    len32 = np.full(1, 32, dtype=np.uint32)

    def single(w):
        s1 = np.zeros(1, dtype=np.uint8)
        for k in range(20):
            i = (w * 131 + k * 17) % NP
            rc = L.hbls_verify_batch(_p(d["pks"][48 * i:]), _p(sigs[96 * i:]), _p(d["item_msgs"][32 * i:]), _p(off0),
                                     _p(len32), 1, _p(s1))
            if rc != 0 or s1[0] != want[i]:
                errs.append((w, i, int(s1[0])))

    ths = [threading.Thread(target=single, args=(w,)) for w in range(8)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    res["single_callers_ok"] = not errs
    res["env"] = {k: v for k, v in os.environ.items() if k.startswith("HBLS_")}
    print(json.dumps(res), flush=True)
    return 0 if all(v for k, v in res.items() if k.endswith("_ok")) else 1


if __name__ == "__main__":
    sys.exit(main())
