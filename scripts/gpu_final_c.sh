#!/bin/bash
# Round-3 final check, part C: the bench lines -- default (C3, every leg), C2, C5, and the native
# partitioned driver at world 1 (RCCL, --force-dist) for C3 and C2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r03final}; mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench_c3.log 2>&1
rc=$?; echo "bench c3 rc=$rc"; grep '^{' $O/bench_c3.log | tail -1 > $O/bench_c3.json; cut -c1-300 $O/bench_c3.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --config c2 > $O/bench_c2.log 2>&1
rc=$?; echo "bench c2 rc=$rc"; grep '^{' $O/bench_c2.log | tail -1 > $O/bench_c2.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --config c5 > $O/bench_c5.log 2>&1
rc=$?; echo "bench c5 rc=$rc"; grep '^{' $O/bench_c5.log | tail -1 > $O/bench_c5.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --config c2 --force-dist --steps 200 --warmup 20 --no-cpu-baseline \
    --no-refstruct > $O/bench_c2_dist1.log 2>&1
rc=$?; echo "bench c2 dist1 rc=$rc"; grep '^{' $O/bench_c2_dist1.log | tail -1 > $O/bench_c2_dist1.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u bench.py --config c3 --force-dist --steps 50 --warmup 20 --no-cpu-baseline \
    --no-refstruct > $O/bench_c3_dist1.log 2>&1
rc=$?; echo "bench c3 dist1 rc=$rc"; grep '^{' $O/bench_c3_dist1.log | tail -1 > $O/bench_c3_dist1.json; [ $rc -ne 0 ] && exit $rc
exit 0
