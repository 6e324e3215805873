#!/usr/bin/env python3
"""Summarise the rocprofv3 passes of tools/gpu.sh pmc: per kernel of the LAST timed slot, the SQ
counters, FETCH_SIZE (x2: gfx950 tallies 128-B requests at 64 B, MI355X_MICROARCH.md 'HBM'),
WRITE_SIZE, and the kernel-trace duration.  Usage: pmc_summary.py <gpurun_out/pmc_TAG> [json]"""
import collections
import csv
import json
import os
import sys


def per_dispatch(path):
    d = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        key = (int(r["Dispatch_Id"]), r["Kernel_Name"].split("(")[0].replace("hb::", "").replace("void ", ""))
        e = d.setdefault(key, {"grid": int(r["Grid_Size"]), "scratch": int(r["Scratch_Size"]),
                               "vgpr": int(r["VGPR_Count"]), "agpr": int(r["Accum_VGPR_Count"])})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return d


def last_by_name(d, n_last=1):
    """The dispatches of the last slot: for each kernel name, its last n_last dispatches."""
    by = collections.defaultdict(list)
    for (i, name), e in d.items():
        by[name].append((i, e))
    return {name: [e for _, e in v[-n_last:]] for name, v in by.items()}


def main():
    root = sys.argv[1]
    sq = per_dispatch(os.path.join(root, "sq", "run_counter_collection.csv"))
    fe = per_dispatch(os.path.join(root, "fetch", "run_counter_collection.csv"))
    wr = per_dispatch(os.path.join(root, "write", "run_counter_collection.csv"))
    stats = {r["Name"].split("(")[0].replace("hb::", ""): r for r in csv.DictReader(open(os.path.join(root, "trace", "run_kernel_stats.csv")))}
    out = {}
    names = collections.OrderedDict()
    for (_, name) in sq:
        names[name] = 1
    # launches per slot of each kernel: the dispatches of the last slot (from its k_attestation_roots
    # to the next message hashing after it, as tools/last_slot.py)
    order = list(sq.keys())
    starts = [k for k, (i, n) in enumerate(order) if n.startswith("k_attestation_roots")]
    slot = order[starts[-1]:] if starts else order
    hashes = [k for k, (i, n) in enumerate(slot) if n.startswith("k_hash_to_g2") or n.startswith("k_h2c_field")]
    slot = slot[:hashes[1]] if len(hashes) > 1 else slot
    slot_names = collections.Counter(n for _, n in slot)
    for name, cnt in slot_names.items():
        S = [sq[k] for k in slot if k[1] == name]
        F = [e for (i, n), e in fe.items() if n == name][-cnt:]
        W = [e for (i, n), e in wr.items() if n == name][-cnt:]
        tot = lambda L, c: sum(e.get(c, 0.0) for e in L)  # noqa: E731
        st = stats.get(name, {})
        out[name] = {
            "launches_per_slot": cnt, "grid": S[0]["grid"], "vgpr": S[0]["vgpr"], "agpr": S[0]["agpr"],
            "scratch_B_per_lane": S[0]["scratch"],
            "SQ_WAVES": tot(S, "SQ_WAVES"), "SQ_INSTS_VALU": tot(S, "SQ_INSTS_VALU"),
            "SQ_INSTS_SALU": tot(S, "SQ_INSTS_SALU"), "SQ_ACTIVE_INST_VALU": tot(S, "SQ_ACTIVE_INST_VALU"),
            "SQ_BUSY_CYCLES": tot(S, "SQ_BUSY_CYCLES"), "SQ_WAVE_CYCLES": tot(S, "SQ_WAVE_CYCLES"),
            "SQ_WAIT_INST_ANY": tot(S, "SQ_WAIT_INST_ANY"), "SQ_WAIT_ANY": tot(S, "SQ_WAIT_ANY"),
            "FETCH_bytes_corrected": 2 * 1024 * tot(F, "FETCH_SIZE"),
            "WRITE_bytes": 1024 * tot(W, "WRITE_SIZE"),
            "trace_avg_ns": float(st["AverageNs"]) if st else None,
        }
    json.dump(out, sys.stdout if len(sys.argv) < 3 else open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
