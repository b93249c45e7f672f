#!/bin/bash
# Per-pair traces of the C3 and C2 early-exit sweeps on the current build (where the time goes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r03n}; mkdir -p $O
for c in c3 c2; do
  timeout -k 10 300 python -u scripts/pair_probe.py $c $O/$c > $O/$c.log 2>&1 || { cat $O/$c.log; exit 1; }
  cat $O/$c.log
  python scripts/pair_trace_summary.py $O/$c.trace > $O/${c}_summary.txt 2>&1; cat $O/${c}_summary.txt
done
