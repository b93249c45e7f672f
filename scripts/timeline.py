"""Kernel timeline of the last launches in a rocprofv3 kernel trace: start offset from the first
shown launch, duration and gap before it (us). Usage: timeline.py kernel_trace.csv [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-n:]
t0 = int(rows[0]["Start_Timestamp"])
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    k = r["Kernel_Name"].split("(")[0].replace("mcmc::", "").replace("void ", "")[:48]
    gap = (s - prev_end) / 1000 if prev_end is not None else 0.0
    print(f"{(s - t0) / 1000:9.2f} {((e - s) / 1000):8.2f} gap {gap:7.2f}  {k}")
    prev_end = e
