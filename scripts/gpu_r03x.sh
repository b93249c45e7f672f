#!/bin/bash
# Wide commit with compact slot headers: wide parity suite, C5 timelines (converged, violator-heavy).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03x}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_wide.py -m gpu -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
Q="--config c5 --steps 20 --warmup 5 --no-cpu-baseline --no-refstruct --no-convergence"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t1 -o run -- python3 bench.py $Q > $O/bench_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
f=$(find $O/t1 -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py $f 8 | head -4
grep '^{' $O/bench_trace.log | tail -1 | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tv -o run -- python3 scripts/c5_viol_probe.py > $O/viol.log 2>&1
rc=$?; echo "viol rc=$rc"; grep rep $O/viol.log
exit $rc
