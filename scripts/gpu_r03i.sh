#!/bin/bash
# r03 records: rocprof kernel stats + PMC passes of the C3 and C5 benches (profiles/r03), the C2
# phase split, the world-1 native-driver bench lines (C2, C3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r03i}
Q="--no-refstruct --no-convergence --no-full-scan"
bash scripts/gpu_prof.sh ${TAG}_c3 $Q || exit $?
bash scripts/gpu_prof.sh ${TAG}_c5 --config c5 $Q || exit $?
O=gpurun_out/$TAG; mkdir -p $O
MCMC_PHASE_DUMP=$O/c2.phase MCMC_PROBE_MODES=0 timeout -k 10 200 python -u scripts/scan_probe.py c2 > $O/c2_phase.log 2>&1
echo "c2 phase rc=$?"; tail -1 $O/c2_phase.log | cut -c1-300
timeout -k 10 300 python -u bench.py --config c2 --force-dist --steps 200 --warmup 10 --no-cpu-baseline \
    --no-refstruct > $O/bench_c2_dist1.log 2>&1
echo "c2 dist rc=$?"; tail -1 $O/bench_c2_dist1.log | cut -c1-300
timeout -k 10 400 python -u bench.py --config c3 --force-dist --steps 30 --warmup 3 --no-cpu-baseline \
    --no-refstruct > $O/bench_c3_dist1.log 2>&1
echo "c3 dist rc=$?"; tail -1 $O/bench_c3_dist1.log | cut -c1-300
timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline --no-refstruct > $O/bench_c2.log 2>&1
echo "c2 rc=$?"; tail -1 $O/bench_c2.log | cut -c1-300
