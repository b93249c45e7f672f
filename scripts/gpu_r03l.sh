#!/bin/bash
# r03 committed profiles: kernel trace + PMC (FETCH_SIZE, WRITE_SIZE) of the C3 and C5 benches at the
# bench's own step counts (50 timed, 5 warmup: the clocks settle over the first ~15 sweeps), then the
# SQ/LDS counter pass of the C3 sweep.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r03l}
Q="--no-refstruct --no-convergence --no-full-scan --steps 50 --warmup 5"
bash scripts/gpu_prof.sh ${TAG}_c3 $Q || exit $?
bash scripts/gpu_prof.sh ${TAG}_c5 --config c5 $Q || exit $?
bash scripts/gpu_pmc_sq.sh ${TAG}_sq
