#!/bin/bash
# r05: the full-size C3 tests (incl. the 252-sweep reference loop vs the streamed restatement) + dense tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r05d}; mkdir -p $O
timeout -k 10 1100 python3 -u -m pytest tests/test_dense.py tests/test_c3_full.py -x -v -s --timeout 900 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|eps |every vertex|Cviol traj|checked" $O/pytest.log | tail -20; tail -2 $O/pytest.log
[ $rc -ne 0 ] && grep -n "Error\|assert" $O/pytest.log | head -30
exit $rc
