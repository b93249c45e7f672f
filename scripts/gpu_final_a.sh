#!/bin/bash
# Round-3 final check, part A: the full-size tests (C3, C4 over 8 loopback ranks, C5 stand-in).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r03final}; mkdir -p $O
for f in c3 c4 c5; do
  timeout -k 10 600 python -u -m pytest tests/test_${f}_full.py -m gpu -x -v -s -p no:cacheprovider --timeout 600 \
      --timeout-method thread > $O/pytest_${f}_full.log 2>&1
  rc=$?; echo "$f full rc=$rc"; tail -3 $O/pytest_${f}_full.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
