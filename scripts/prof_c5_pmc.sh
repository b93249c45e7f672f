#!/bin/bash
# C5 (wide sweep) HBM traffic: rocprofv3 FETCH_SIZE and WRITE_SIZE in separate passes, plus a kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_c5pmc
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --config c5 --steps 20 --warmup 2 --no-cpu-baseline --no-refstruct > $OUT/bench_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -1 $OUT/bench_trace.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc1 -o run -- python3 bench.py --config c5 --steps 8 --warmup 1 --no-cpu-baseline --no-refstruct > $OUT/bench_pmc1.log 2>&1
rc=$?; echo "pmc1 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc2 -o run -- python3 bench.py --config c5 --steps 8 --warmup 1 --no-cpu-baseline --no-refstruct > $OUT/bench_pmc2.log 2>&1
rc=$?; echo "pmc2 rc=$rc"
find $OUT -name "*.csv" | head
exit $rc
