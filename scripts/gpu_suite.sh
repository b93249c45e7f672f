#!/bin/bash
# the whole -m gpu suite (as the driver runs it), log under gpurun_out/<tag>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-suite}; mkdir -p $O
shift
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider "$@" > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -ne 0 ] && grep -n "Error\|assert\|FAIL" $O/pytest.log | head -30
exit $rc
