#!/bin/bash
# r03: full-size checks -- C3 every vertex (two eps), C4 loopback world 8 (equal / unequal plans, delta
# exchange and its overflow fallback).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03b}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_c3_full.py tests/test_c4_full.py -m gpu -x -v -s -p no:cacheprovider \
    --timeout 900 --timeout-method thread > $OUT/pytest_full.log 2>&1
rc=$?; echo "full rc=$rc"; grep -E "PASS|FAIL|Error|C4 loop|every vertex|changed|C3 graph" $OUT/pytest_full.log | tail -20
exit $rc
