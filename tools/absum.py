#!/usr/bin/env python3
"""Summary of A/B bench results (bench_<variant>_<k>.json): per variant the value, ms/step, parity, selected kernel
times and the single-call latency.  Usage: absum.py TAG"""
import json
import os
import sys

tag = sys.argv[1]
k = 1
while os.path.exists(f"gpurun_out/ab_{tag}_{k}.json"):
    env = open(f"gpurun_out/ab_{tag}_{k}.env").read().strip() if os.path.exists(f"gpurun_out/ab_{tag}_{k}.env") else "?"
    try:
        d = json.loads(open(f"gpurun_out/ab_{tag}_{k}.json").read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(k, env, "unreadable", e)
        k += 1
        continue
    ks = d.get("kernels", {})
    cc = d.get("concurrent_callers") or {}
    sel = {n: ks[n]["ms_per_step"] for n in ("k_pair3_mml", "k_pair3_fin", "k_pair3_ml", "k_pair3_mls", "k_slines",
                                            "k_dec_sig_pt", "k_hash_to_g2", "k_rlc", "k_ta_small") if n in ks}
    print(k, env.replace("HBLS_LIBRARY=charon_amd/lib/variants/", "")[:60], d["value"], d["ms_per_step"],
          all(d["parity"].values()), sel, cc.get("single_call_latency_ms"), cc.get("calls_per_s"))
    if cc.get("single_call_kernels_ms"):
        print("   single call:", cc["single_call_kernels_ms"])
    k += 1
