#!/bin/bash
# r03 first GPU pass: partitioned-path tests, RCCL multi-process worlds, C3/C2 pair traces,
# world-1 native-driver bench lines (C2, C3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03a}
mkdir -p $OUT
timeout -k 10 300 python -u scripts/pair_probe.py c3 $OUT/c3 > $OUT/pair_c3.log 2>&1
echo "pair c3 rc=$?"; tail -2 $OUT/pair_c3.log
timeout -k 10 200 python -u scripts/pair_probe.py c2 $OUT/c2 > $OUT/pair_c2.log 2>&1
echo "pair c2 rc=$?"; tail -2 $OUT/pair_c2.log
timeout -k 10 600 python -u -m pytest tests/test_multi.py tests/test_cli.py -m gpu -x -v -p no:cacheprovider \
    --timeout 240 --timeout-method thread > $OUT/pytest_multi.log 2>&1
rc=$?; echo "multi rc=$rc"; tail -5 $OUT/pytest_multi.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_rccl_world.py -m gpu -x -v -p no:cacheprovider \
    --timeout 280 --timeout-method thread > $OUT/pytest_rccl.log 2>&1
rc=$?; echo "rccl rc=$rc"; tail -5 $OUT/pytest_rccl.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --config c2 --force-dist --steps 200 --warmup 10 --no-cpu-baseline \
    --no-refstruct > $OUT/bench_c2_dist1.log 2>&1
echo "c2 dist rc=$?"; tail -1 $OUT/bench_c2_dist1.log | cut -c1-300
timeout -k 10 400 python -u bench.py --config c3 --force-dist --steps 30 --warmup 3 --no-cpu-baseline \
    --no-refstruct > $OUT/bench_c3_dist1.log 2>&1
echo "c3 dist rc=$?"; tail -1 $OUT/bench_c3_dist1.log | cut -c1-300
