#!/usr/bin/env python3
"""GPU diagnosis: the host-buffer Verify and ThresholdAggregate batches on a C5-style shard (1 %
of the partials corrupted in fifths, bench.corrupt), two Verify calls in a row (the first takes
the slot-wide check, the second -- adaptive -- the per-batch check directly), each compared with
the statuses expected by construction.  Usage: diag_c5_host.py [validators]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (HIP runtime first, as bench.py)

import bench  # noqa: E402
from charon_amd import _lib  # noqa: E402

V = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
L = _lib.load_library()
bench._chk(L, L.hbls_init(0))
wl = bench.WORKLOADS["c5"]
d = bench.setup_inputs(L, wl, V, 0)
bench.corrupt(L, d, wl["adversarial"], 7)
NP = d["NP"]
exp_v = d["exp_v"]
for call in range(3):
    st = np.full(NP, 255, dtype=np.uint8)
    bench._chk(L, L.hbls_verify_batch(bench._p(d["pks"]), bench._p(d["sigs"]), bench._p(d["item_msgs"]),
                                      bench._p(d["item_off"]), bench._p(d["item_len"]), NP, bench._p(st)))
    bad = np.nonzero(st != exp_v)[0]
    print("verify call", call, "mismatches", len(bad), "examples", [(int(i), int(st[i]), int(exp_v[i])) for i in bad[:10]],
          flush=True)
tout = np.zeros(V * 96, dtype=np.uint8)
tst = np.zeros(V, dtype=np.uint8)
bench._chk(L, L.hbls_threshold_aggregate_batch(bench._p(d["ta_sigs"]), bench._p(d["ta_idx"]), bench._p(d["grp_off"]),
                                               V, bench._p(tout), bench._p(tst)))
badt = np.nonzero(tst != d["exp_ta"])[0]
clean = d["exp_agg"] == 0
bada = np.nonzero(~np.all(tout.reshape(V, 96)[clean] == d["root_sigs"].reshape(V, 96)[clean], axis=1))[0]
print("ta status mismatches", len(badt), [(int(i), int(tst[i]), int(d["exp_ta"][i])) for i in badt[:10]])
print("ta aggregate mismatches among clean", len(bada))
