#!/bin/bash
# One GPU check of the round: the full-size C3 test, the GPU suite, smoke(), the default bench line.
# Stops at the first failing step. Usage: scripts/gpu_round.sh [TAG] [extra pytest args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r02}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_c3_full.py -m gpu -x -v -s -p no:cacheprovider --timeout 600 \
    --timeout-method thread > $OUT/pytest_c3_full.log 2>&1
rc=$?; echo "c3 full rc=$rc"; tail -12 $OUT/pytest_c3_full.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    --deselect tests/test_c3_full.py "$@" > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u bench.py > $OUT/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench_default.log | cut -c1-3000
exit $rc
