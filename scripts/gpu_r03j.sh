#!/bin/bash
# r03: GPU suite (minus the full-size checks), world-1 native-driver benches, default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r03j}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    --deselect tests/test_c3_full.py --deselect tests/test_c4_full.py --deselect tests/test_c5_full.py > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --config c2 --force-dist --steps 200 --warmup 10 --no-cpu-baseline \
    --no-refstruct > $O/bench_c2_dist1.log 2>&1
echo "c2 dist rc=$?"; tail -1 $O/bench_c2_dist1.log | cut -c1-250
timeout -k 10 400 python -u bench.py --config c3 --force-dist --steps 50 --warmup 3 --no-cpu-baseline \
    --no-refstruct > $O/bench_c3_dist1.log 2>&1
echo "c3 dist rc=$?"; tail -1 $O/bench_c3_dist1.log | cut -c1-250
timeout -k 10 600 python -u bench.py --no-refstruct --no-cpu-baseline > $O/bench_c3.log 2>&1
echo "bench rc=$?"; tail -1 $O/bench_c3.log | cut -c1-250
timeout -k 10 300 python -u bench.py --config c5 --no-refstruct --no-cpu-baseline > $O/bench_c5.log 2>&1
echo "c5 rc=$?"; tail -1 $O/bench_c5.log | cut -c1-250
