"""Mean/median duration (us) per kernel over the last N launches of a rocprofv3 kernel trace."""
import csv
import statistics
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 60
d = defaultdict(list)
for r in rows:
    k = r['Kernel_Name'].split('(')[0].replace('mcmc::', '').replace('void ', '').split('<')[0]
    d[k].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000)
for k, v in d.items():
    v = v[-last:]
    if len(v) >= 5:
        print(f"{k[:40]:40s} n={len(v):4d} mean {statistics.mean(v):8.2f} median {statistics.median(v):8.2f} max {max(v):8.2f}")
