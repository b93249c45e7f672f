#!/bin/bash
# Fast wide commit with the walks' events sorted in LDS: wide parity + full-size C5, violator loop, C5 line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03af}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_wide.py tests/test_c5_full.py -m gpu -x -q -p no:cacheprovider \
    --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 scripts/c5_viol_probe.py > $O/viol_$i.log 2>&1 || exit $?
  echo "$(grep rep $O/viol_$i.log | tr '\n' ' ' | cut -c1-200)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tv -o run -- python3 scripts/c5_viol_probe.py > $O/viol_t.log 2>&1 || exit $?
python3 scripts/viol_trace.py $(find $O/tv -name "*kernel_trace.csv" | head -1) 12
