#!/bin/bash
# C5 kernel timeline with the incremental wide sweep (and without), short bench legs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03p}; mkdir -p $O
Q="--config c5 --steps 20 --warmup 5 --no-cpu-baseline --no-refstruct --no-convergence"
for m in 1 0; do
  MCMC_WIDE_INC=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$m -o run -- python3 bench.py $Q > $O/bench$m.log 2>&1
  rc=$?; echo "trace inc=$m rc=$rc"; [ $rc -ne 0 ] && exit $rc
  f=$(find $O/t$m -name "*kernel_trace.csv" | head -1)
  python3 scripts/timeline.py $f 24
  python3 scripts/trace_avg.py $f 40
done
