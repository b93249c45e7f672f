#!/bin/bash
# rocprofv3 kernel trace of the c5 bench (wide sweep) -- per-kernel durations.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-c5}; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --config c5 --steps 20 --warmup 2 --no-cpu-baseline --no-refstruct "$@" > $OUT/bench_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -1 $OUT/bench_trace.log | cut -c1-400
find $OUT -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-250 | head -30
exit $rc
