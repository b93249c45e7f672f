#!/bin/bash
# Violator-heavy C5 sweeps (nCol = maxDeg / 4): kernel timeline of the reference loop (2 reps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03v}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- python3 scripts/c5_viol_probe.py > $O/probe.log 2>&1
rc=$?; echo "probe rc=$rc"; cat $O/probe.log | grep rep; [ $rc -ne 0 ] && exit $rc
f=$(find $O/t -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py $f 22
