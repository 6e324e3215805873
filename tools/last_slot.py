#!/usr/bin/env python3
"""Per-kernel durations of the LAST slot in a rocprofv3 kernel trace of bench.py: the serialised
roofline slot that bench.py runs after its timed region (library timing mode 2), to compare with
the bench line's `kernels` (alone) figures.  Usage: last_slot.py run_kernel_trace.csv"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_attestation_roots" in r["Kernel_Name"]]
last = rows[starts[-1]:] if starts else rows
# the serialised slot ends where bench.py's later measurements begin (their first message hashing)
hashes = [i for i, r in enumerate(last) if "k_hash_to_g2" in r["Kernel_Name"] or "k_h2c_field" in r["Kernel_Name"]]
last = last[:hashes[1]] if len(hashes) > 1 else last
tot = collections.OrderedDict()
for r in last:
    n = r["Kernel_Name"].split("(")[0].replace("hb::", "")
    tot[n] = tot.get(n, 0.0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
print("kernel                      ms (sum of the last slot's launches, from the trace)")
for n, ms in tot.items():
    print("%-26s %10.3f" % (n, ms))
