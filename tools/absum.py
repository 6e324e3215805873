#!/usr/bin/env python3
"""Summary of tools/gpu.sh ab results: gpurun_out/ab_TAG_WORKLOAD_LABEL_REP.json -> per run the value,
ms/step, single-call latency and the kernels' alone times.  Usage: absum.py TAG [kernel substrings]"""
import glob
import json
import sys

tag = sys.argv[1]
keys = sys.argv[2:] or ["hash", "lines", "pair3", "lml", "fin", "dec", "rlc", "ta_small", "slines", "fb"]
for f in sorted(glob.glob(f"gpurun_out/ab_{tag}_*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable", e)
        continue
    ks = {n: round(v["ms_per_step"], 2) for n, v in d.get("kernels", {}).items()
          if isinstance(v, dict) and "ms_per_step" in v and any(k in n for k in keys)}
    lat = d.get("single_call_latency_ms")
    cc = (d.get("concurrent_callers") or {}).get("calls_per_s")
    print(f.split("/")[-1][len("ab_"):-5], f"{d['value'] / 1e6:.3f} M/s", f"{d['ms_per_step']:.2f} ms",
          f"lat {lat}" if lat else "", f"callers {cc}" if cc else "", ks)
