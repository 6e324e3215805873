#!/usr/bin/env python3
"""Print the kernel timeline of the last N slots (or single calls) of a rocprofv3 kernel trace
(tools/gpu.sh trace / single).  Usage: timeline.py run_kernel_trace.csv [N [min_ms]]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 2
idx = [i for i, r in enumerate(rows) if "k_hash_to_g2" in r["Kernel_Name"] or "k_h2c_field" in r["Kernel_Name"]]
sl = rows[idx[-n]:]
t0 = int(sl[0]["Start_Timestamp"])
for r in sl:
    name = r["Kernel_Name"].split("(")[0].replace("hb::", "")
    s = (int(r["Start_Timestamp"]) - t0) / 1e6
    e = (int(r["End_Timestamp"]) - t0) / 1e6
    if e - s > float(sys.argv[3] if len(sys.argv) > 3 else 0.05):
        print("%-22s q%-3s %8.2f %8.2f %8.2f grid=%s" % (name[:22], r["Queue_Id"], s, e, e - s, r["Grid_Size_X"]))
