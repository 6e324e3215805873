#!/usr/bin/env python3
"""One-screen summary of bench.py JSON lines (the last line of each file): value, ms/step, parity,
per-kernel alone times.  Usage: bsum.py FILE..."""
import json
import sys

for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], all(d["parity"].values()))
    kt = d.get("with_key_tables") or {}
    print("  key tables:", kt.get("items_per_s"), kt.get("ms_per_step"))
    print("  " + "  ".join(f"{k}={v['ms_per_step']}" for k, v in d.get("kernels", {}).items()))
    r = d.get("roofline") or {}
    print("  roofline:", r.get("kernel"), r.get("frac"), (r.get("slot") or {}).get("frac"))
