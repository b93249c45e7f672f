#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench, then PMC HBM counters in separate passes
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950). Extra args go to bench.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r01}; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline "$@" > $OUT/bench_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -1 $OUT/bench_trace.log | cut -c1-300
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc1 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > $OUT/bench_pmc1.log 2>&1
rc=$?; echo "pmc1 rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc2 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > $OUT/bench_pmc2.log 2>&1
rc=$?; echo "pmc2 rc=$rc"
find $OUT -name "*.csv" | head -20
exit $rc
