"""Print one slot's kernel timeline from a rocprofv3 kernel trace: python tools/timeline.py <run_kernel_trace.csv>"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_hash_to_g2" in r["Kernel_Name"]]
i0 = idx[-2]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:idx[-1]]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{r['Kernel_Name'][:28]:30s} q{r.get('Queue_Id', '?'):>3} start {s / 1e6:8.3f}  end {e / 1e6:8.3f}  dur {(e - s) / 1e6:7.3f}")
