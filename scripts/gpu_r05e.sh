#!/bin/bash
# r05: the wide sweep over the tiled layout (small-graph parity, then C3 at nCol = maxDeg)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r05e}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_wide.py -k "wide_tiled or generated" -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/small.log 2>&1
rc=$?; grep -E "PASS|FAIL" $O/small.log | tail -30; tail -2 $O/small.log
if [ $rc -ne 0 ]; then grep -n "Error\|assert" $O/small.log | head -30; exit $rc; fi
timeout -k 10 1150 python3 -u -m pytest tests/test_c3_full.py -k default_ncol -x -v -s --timeout 1100 --timeout-method thread -p no:cacheprovider > $O/c3.log 2>&1
rc=$?; grep -E "PASS|FAIL|nCol|Cviol traj|checked" $O/c3.log | tail -20; tail -2 $O/c3.log
[ $rc -ne 0 ] && grep -n "Error\|assert" $O/c3.log | head -30
exit $rc
