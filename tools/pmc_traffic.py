#!/usr/bin/env python3
"""profiles/pmc_traffic.json from a tools/pmc_summary.py summary: HBM bytes per slot (FETCH_SIZE
doubled per MI355X_MICROARCH.md, WRITE_SIZE, KB -> bytes) under the names bench.py times the
kernels by (hipbls.hip TIMED labels), summed over the kernels behind each label.
Usage: pmc_traffic.py profiles/<tag>_pmc_summary.json <tag>"""
import json
import sys

LABELS = {  # bench.py / TIMED label -> kernel symbols of the slot
    "k_hash_to_g2": ["k_hash_to_g2_1", "k_hash_to_g2", "k_h2c_field", "k_h2c_map", "k_h2c_clear1", "k_h2c_clear1b",
                     "k_h2c_clear2", "k_h2c_clear3", "k_h2c_clear1h", "k_h2c_clear2h"], "k_lines_msg": ["k_lines_msg"],
    "k_dec_pk": ["k_dec_pk", "k_g1_subgroup"], "k_dec_sig_pt": ["k_dec_sig_pt", "k_g2_subgroup"], "k_ta_straus": ["k_ta_jtab", "k_ta_jladder", "k_ta_jgeneral", "k_ta_joint", "k_ta_straus"],
    "k_ta_small": ["k_ta_sprep", "k_ta_small", "k_ta_stab", "k_ta_sladder", "k_ta_sladder<false>", "k_ta_sladder<true>"], "k_mml_eval": ["k_mml_eval"],
    "k_pair3_mls": ["k_pair3<5>", "k_lml<0>", "k_lml<1>"],
    "k_group_sum": ["k_group_sum"], "k_rlc": ["k_rlc_msm<1>", "k_rlc<1>", "k_rlc_msm<2>", "k_rlc<2>", "k_rlc_msm<3>", "k_rlc<3>", "k_rlc_msm", "k_rlc",
              "k_rlc_msm<1, 0>", "k_rlc_msm<1, 1>", "k_rlc_msm<1, 2>", "k_rlc_msm<2, 0>", "k_rlc_msm<2, 1>",
              "k_rlc_msm<2, 2>", "k_rlc_msm<3, 0>", "k_rlc_msm<3, 1>"], "k_group_prep": ["k_group_prep_p", "k_group_prep_b"],
    "k_msm_bucket": ["k_msm_bucket"], "k_msm_reduce": ["k_msm_reduce"], "k_msm_sum": ["k_msm_sum"],
    "k_slines": ["k_slines"], "k_lines_at_p": ["k_lines_at_p"], "k_pair3_mml": ["k_pair3<4>"], "k_pair3_prod": ["k_pair3<3>"],
    "k_pair3_fin": ["k_pair3<2>", "k_pair6_fin", "k_pair6_fin<3>", "k_pair6_fin<10>"], "k_pair3_ml": ["k_pair3<1>"], "k_attestation_roots": ["k_attestation_roots"],
}

s = json.load(open(sys.argv[1]))
out = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over one C3 slot (tools/gpu.sh pmc {sys.argv[2]}; "
                 "FETCH_SIZE doubled per MI355X_MICROARCH.md, KB -> bytes): bytes per slot of each timed kernel "
                 "label (all its launches, as bench.py's per-kernel times)", "kernels": {}}
for label, syms in LABELS.items():
    es = [s[k] for k in syms if k in s]
    if not es:
        continue
    f = sum(e["FETCH_bytes_corrected"] for e in es)
    w = sum(e["WRITE_bytes"] for e in es)
    out["kernels"][label] = {"bytes_per_slot": f + w, "fetch": f, "write": w,
                             "launches_per_slot": sum(e["launches_per_slot"] for e in es),
                             "scratch_B_per_lane": max(e["scratch_B_per_lane"] for e in es),
                             "valu_wave_insts": sum(e["SQ_INSTS_VALU"] for e in es)}
json.dump(out, open("profiles/pmc_traffic.json", "w"), indent=1)
print(json.dumps({k: round(v["bytes_per_slot"] / 1e9, 2) for k, v in out["kernels"].items()}))
