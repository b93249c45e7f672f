#!/bin/bash
# Tiled sweep prologue (first-row bounds and group powers beside the state words; no post-arrival
# state load without events): tiled parity + partitioned suites, full-size C3, C2 / C3 bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r03ac}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_multi.py tests/test_c3_full.py -m gpu -x -q \
    -p no:cacheprovider --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
Q="--no-refstruct --no-convergence --no-cpu-baseline --no-full-scan"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config c2 $Q > $O/bench_c2_$i.log 2>&1
  rc=$?; echo "c2 $i rc=$rc $(tail -1 $O/bench_c2_$i.log | cut -c150-215)"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 600 python -u bench.py $Q > $O/bench_c3.log 2>&1
rc=$?; echo "c3 rc=$rc $(tail -1 $O/bench_c3.log | cut -c150-215)"
exit $rc
