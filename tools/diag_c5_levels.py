#!/usr/bin/env python3
"""GPU diagnosis: the C4 shard with 1 % of the partials corrupted, one corruption class at a time
(bench.corrupt classes), two slot calls (the second behind the adaptive switch, i.e. the per-batch
check); prints the library's fallback counters per class next to the groups that fail by
construction.  Usage: HBLS_STATS=1 diag_c5_levels.py [classes...]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import bench  # noqa: E402
from charon_amd import _lib  # noqa: E402
from test_gpu_configs import _run_slot  # noqa: E402

L = _lib.load_library()
wl = bench.WORKLOADS["c4"]
base = bench.setup_inputs(L, wl, wl["validators"], 0)
OK, NV = 0, 3


def stats():
    st = (ctypes.c_uint64 * 6)()
    L.hbls_stats(st, 6)
    return list(st)


for c in [int(x) for x in sys.argv[1:]] or [0, 1, 2, 3, 4]:
    d = dict(base)
    d["sigs"] = base["sigs"].copy()
    bench.corrupt(L, d, 0.01, seed=7, classes=(c,))
    n, V = d["n"], d["V"]
    bad_groups = set(int(i) // n for i in np.nonzero(d["exp_v"] == NV)[0])
    bad_groups |= set(int(v) for v in np.nonzero(d["exp_agg"] == NV)[0])
    for k in range(2):
        s0 = stats()
        vst, tst, ast, tout = _run_slot(L, d, sigs=d["sigs"])
        s1 = stats()
        exact = bool((vst == d["exp_v"]).all() and (ast == d["exp_agg"]).all())
        print(f"class {c} call {k}: corrupted {d['n_corrupted']}, groups failing by construction {len(bad_groups)}, "
              f"fallback items {s1[2] - s0[2]}, groups in failing batches {s1[3] - s0[3]}, exact {exact}",
              flush=True)
