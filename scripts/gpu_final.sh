#!/bin/bash
# Final records of a round: rocprof kernel stats + PMC passes of the C3 and C5 benches, then the full
# default (C3) and C5 bench lines. Usage: scripts/gpu_final.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-final}
Q="--no-refstruct --no-convergence --no-full-scan"
bash scripts/gpu_prof.sh ${TAG}_c3 $Q || exit $?
bash scripts/gpu_prof.sh ${TAG}_c5 --config c5 $Q || exit $?
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench_c3_default.log 2>&1 || exit $?
echo "c3 $(tail -1 $O/bench_c3_default.log | cut -c1-300)"
timeout -k 10 600 python -u bench.py --config c5 > $O/bench_c5.log 2>&1 || exit $?
echo "c5 $(tail -1 $O/bench_c5.log | cut -c1-300)"
