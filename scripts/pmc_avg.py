"""Average rocprofv3 --pmc counter values per dispatch of the kernels whose name contains a substring."""
import csv
import sys
from collections import defaultdict
from pathlib import Path

root, sub = Path(sys.argv[1]), sys.argv[2]
vals = defaultdict(list)
for f in root.rglob("*counter_collection.csv"):
    for row in csv.DictReader(open(f)):
        if sub in row.get("Kernel_Name", ""):
            vals[(row["Kernel_Name"][:60], row["Counter_Name"])].append(float(row["Counter_Value"]))
for (k, c), v in sorted(vals.items()):
    print(f"{k:60s} {c:24s} n={len(v):4d} avg={sum(v) / len(v):.4g}")
