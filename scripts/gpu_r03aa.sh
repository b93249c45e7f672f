#!/bin/bash
# Pipelined walks: wide parity suite, full-size C5 check, violator-heavy loop timeline, C5 timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03aa}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_wide.py -m gpu -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_c5_full.py -m gpu -x -q -s -p no:cacheprovider \
    --timeout 600 --timeout-method thread > $O/pytest_c5_full.log 2>&1
rc=$?; echo "c5 full rc=$rc"; tail -2 $O/pytest_c5_full.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tv -o run -- python3 scripts/c5_viol_probe.py > $O/viol.log 2>&1
rc=$?; echo "viol rc=$rc"; grep rep $O/viol.log; [ $rc -ne 0 ] && exit $rc
python3 scripts/viol_trace.py $(find $O/tv -name "*kernel_trace.csv" | head -1) 12
