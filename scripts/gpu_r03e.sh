#!/bin/bash
# r03: C3/C2 traces (pairs + tail queue) and the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03e}
mkdir -p $OUT
timeout -k 10 300 python -u scripts/pair_probe.py c3 $OUT/c3 > $OUT/pair_c3.log 2>&1
echo "pair c3 rc=$?"; tail -1 $OUT/pair_c3.log
timeout -k 10 200 python -u scripts/pair_probe.py c2 $OUT/c2 > $OUT/pair_c2.log 2>&1
echo "pair c2 rc=$?"; tail -1 $OUT/pair_c2.log
timeout -k 10 600 python -u bench.py --no-refstruct --no-cpu-baseline > $OUT/bench_c3.log 2>&1
echo "bench rc=$?"; tail -1 $OUT/bench_c3.log | cut -c1-600
