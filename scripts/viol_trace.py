"""Kernel durations of the sweeps after the last colouring init in a rocprofv3 kernel trace (the
violator-heavy C5 loop of c5_viol_probe.py). Usage: viol_trace.py kernel_trace.csv [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
sel = [r for r in rows if any(k in r["Kernel_Name"] for k in ("wide_", "commit", "init_coloring"))]
starts = [i for i, r in enumerate(sel) if "init_coloring" in r["Kernel_Name"]]
sel = sel[starts[-1] + 1:starts[-1] + 1 + n] if starts else sel[-n:]
t0 = int(sel[0]["Start_Timestamp"])
for r in sel:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1000:9.2f} {(e - s) / 1000:8.2f}  {r['Kernel_Name'].split('(')[0].replace('mcmc::', '')[:44]}")
