#!/bin/bash
# C2 late staging: tiled parity + multi suites, A/B of MCMC_LATE_STAGE on the C2 probe (alternating),
# then the C2 and C3 bench lines (short legs only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r03m}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_multi.py tests/test_c3_full.py -m gpu -x -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for L in 0 1; do
    MCMC_LATE_STAGE=$L MCMC_PROBE_MODES=0 timeout -k 10 300 python -u scripts/scan_probe.py c2 > $O/c2_L${L}_$i.log 2>&1 || exit $?
    echo "L$L/$i $(grep '^{' $O/c2_L${L}_$i.log | cut -c1-200)"
  done
done
Q="--no-refstruct --no-convergence --no-cpu-baseline"
timeout -k 10 600 python -u bench.py --config c2 $Q > $O/bench_c2.log 2>&1
rc=$?; echo "bench c2 rc=$rc"; tail -1 $O/bench_c2.log | cut -c1-1500; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py $Q --no-full-scan > $O/bench_c3.log 2>&1
rc=$?; echo "bench c3 rc=$rc"; tail -1 $O/bench_c3.log | cut -c1-800
exit $rc
