#!/bin/bash
# C5 (configs[4] stand-in): R-MAT generator parity, wide-sweep parity, then the c5 bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rmat.py tests/test_wide.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c5_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -25 gpurun_out/c5_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --config c5 --steps 20 --warmup 3 "$@" > gpurun_out/bench_c5.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_c5.log | cut -c1-3000
exit $rc
