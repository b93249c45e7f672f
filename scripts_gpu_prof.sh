#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench, then PMC HBM counters in separate passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${1:-r01}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > $OUT/bench_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -3 $OUT/bench_trace.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc1 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_pmc1.log 2>&1
rc=$?; echo "pmc1 rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc2 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_pmc2.log 2>&1
rc=$?; echo "pmc2 rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAVES --output-format csv -d $OUT/pmc3 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_pmc3.log 2>&1
rc=$?; echo "pmc3 rc=$rc"
find $OUT -name "*.csv" | head -20
exit $rc
