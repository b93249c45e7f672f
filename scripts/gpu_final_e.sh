#!/bin/bash
# Round-3 final check, part E: the C5 bench line again, reading the refreshed PMC summary.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r03final}; mkdir -p $O
timeout -k 10 600 python -u bench.py --config c5 > $O/bench_c5_e.log 2>&1
rc=$?; echo "bench c5 rc=$rc"; grep '^{' $O/bench_c5_e.log | tail -1 > $O/bench_c5_e.json; cut -c1-200 $O/bench_c5_e.json
exit $rc
