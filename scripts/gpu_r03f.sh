#!/bin/bash
# r03: traces, the sweep parity suites, the full-size C3/C4 checks, the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03f}
mkdir -p $OUT
timeout -k 10 300 python -u scripts/pair_probe.py c3 $OUT/c3 > $OUT/pair_c3.log 2>&1
echo "pair c3 rc=$?"; tail -1 $OUT/pair_c3.log
timeout -k 10 200 python -u scripts/pair_probe.py c2 $OUT/c2 > $OUT/pair_c2.log 2>&1
echo "pair c2 rc=$?"; tail -1 $OUT/pair_c2.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_multi.py -m gpu -x -q -p no:cacheprovider \
    --timeout 240 --timeout-method thread > $OUT/pytest_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 $OUT/pytest_parity.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 1000 python -u -m pytest tests/test_c3_full.py tests/test_c4_full.py tests/test_c5_full.py -m gpu -x -v -s -p no:cacheprovider \
    --timeout 900 --timeout-method thread > $OUT/pytest_full.log 2>&1
rc=$?; echo "full rc=$rc"; grep -E "PASS|FAIL|Error|every vertex|changed|C5|C4 loop" $OUT/pytest_full.log | tail -12
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --no-refstruct --no-cpu-baseline > $OUT/bench_c3.log 2>&1
echo "bench rc=$?"; tail -1 $OUT/bench_c3.log | cut -c1-400
