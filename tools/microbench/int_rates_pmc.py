#!/usr/bin/env python3
"""Pin the roofline peak from counters: join the int_rates microbenchmark's own lines with a
rocprofv3 kernel trace and one PMC pass of the same binary.

    rocprofv3 --kernel-trace -d D/trace -o run --output-format csv -- ./int_rates > D/int_rates.txt
    rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d D/pmc -o run --output-format csv -- ./int_rates
    int_rates_pmc.py D > profiles/<round>_peak_from_counters.json

Per timed dispatch (the second launch of each kernel and occupancy; the first is the warm-up):
  * VALU instructions per wave (SQ_INSTS_VALU / SQ_WAVES) against the copies the kernel issues
    (ITERS x UNROLL, plus the few outside the loop): a rate above 64 lane-ops/clk/CU with the
    expected count means the instruction dual-issues, with a higher count the accounting is wrong;
  * the effective clock, GRBM_GUI_ACTIVE (busy cycles, summed over the eight XCDs' GRBMs) / 8 over
    the dispatch's duration in the kernel trace, against the in-kernel clock the binary prints;
  * lane-ops/s from counters: SQ_INSTS_VALU x 64 / duration -- for v_mad_u64_u32 at 16 waves per
    CU this must reproduce opcounts.PEAK_MAD_TOPS (32.654 T) within 3 %.
"""
import collections
import csv
import json
import os
import re
import sys

NAMES = {"k_mad64": "v_mad_u64_u32", "k_mullo": "v_mul_lo_u32", "k_mulhi": "v_mul_hi_u32", "k_add": "v_add_u32",
         "k_add3": "v_add3_u32", "k_and": "v_and_b32", "k_mad24": "v_mad_u32_u24", "k_lshr64": "v_lshrrev_b64",
         "k_lshladd64": "v_lshl_add_u64", "k_fma64": "v_fma_f64"}


XCDS = 8  # MI355X: 8 XCDs x 32 CUs


def _kname(s):
    return s.split("(")[0].replace("void ", "").strip()


def main():
    root = sys.argv[1]
    trace = [r for r in csv.DictReader(open(os.path.join(root, "trace", "run_kernel_trace.csv")))]
    pmc = collections.OrderedDict()
    for r in csv.DictReader(open(os.path.join(root, "pmc", "run_counter_collection.csv"))):
        key = (int(r["Dispatch_Id"]), _kname(r["Kernel_Name"]))
        pmc.setdefault(key, {})[r["Counter_Name"]] = pmc.get(key, {}).get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    # the binary's own lines: (waves/CU, instruction) -> (T lane-ops/s, eff MHz)
    own = {}
    for line in open(os.path.join(root, "int_rates.txt")):
        m = re.match(r"waves/CU\s+(\d+)\s+(\S+)\s+([\d.]+) T lane-ops/s\s+([\d.]+) ms\s+eff clock\s+(\d+) MHz", line)
        if m:
            own[(int(m.group(1)), m.group(2))] = {"T_lane_ops": float(m.group(3)), "ms": float(m.group(4)),
                                                  "eff_MHz": float(m.group(5))}
    copies = int(os.environ.get("INT_RATES_COPIES", 16384 * 16))
    # dispatches in launch order: per kernel name, warm-up then timed, for 8 then 16 waves per CU
    tr = collections.defaultdict(list)
    for r in trace:
        tr[_kname(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    pm = collections.defaultdict(list)
    for (i, name), c in pmc.items():
        pm[name].append(c)
    out = {"copies_per_wave": copies, "kernels": []}
    for kname, instr in NAMES.items():
        for j, wpc in enumerate((8, 16)):
            if len(tr[kname]) < 2 * j + 2 or len(pm[kname]) < 2 * j + 2:
                continue
            dur = tr[kname][2 * j + 1]
            c = pm[kname][2 * j + 1]
            waves = c.get("SQ_WAVES", 0.0)
            valu = c.get("SQ_INSTS_VALU", 0.0)
            gui = c.get("GRBM_GUI_ACTIVE", 0.0)
            e = {"instruction": instr, "waves_per_cu": wpc, "duration_ms_trace": round(dur * 1e3, 4),
                 "valu_per_wave": round(valu / waves, 1) if waves else None,
                 "valu_lane_ops_T_from_counters": round(valu * 64 / dur / 1e12, 3) if dur else None,
                 "grbm_gui_active": gui,
                 # one GRBM per XCD: the counter sums the eight XCDs' busy cycles
                 "clock_MHz_from_grbm": round(gui / XCDS / dur / 1e6, 1) if dur else None,
                 **{f"binary_{k}": v for k, v in own.get((wpc, instr), {}).items()}}
            out["kernels"].append(e)
    mad = [k for k in out["kernels"] if k["instruction"] == "v_mad_u64_u32" and k["waves_per_cu"] == 16]
    if mad:
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
        from charon_amd import opcounts
        got = mad[0]["valu_lane_ops_T_from_counters"]
        out["peak_check"] = {"PEAK_MAD_TOPS": opcounts.PEAK_MAD_TOPS, "from_counters": got,
                             "ratio": round(got / opcounts.PEAK_MAD_TOPS, 4) if got else None}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
