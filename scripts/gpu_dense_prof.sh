#!/bin/bash
# dense tests, then the dense-sweep profiles (profiles/r04/) (trace + FETCH/WRITE for c3, c2, c5) and bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-dense_prof}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dense.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/dense.log 2>&1 || { echo "dense rc=$?"; tail -30 $O/dense.log; exit 1; }
tail -1 $O/dense.log
Q="--no-refstruct --no-convergence --no-full-scan --no-cpu-baseline"
bash scripts/gpu_prof.sh ${1:-r04}_c3 $Q || exit $?
bash scripts/gpu_prof.sh ${1:-r04}_c2 --config c2 $Q || exit $?
bash scripts/gpu_prof.sh ${1:-r04}_c5 --config c5 $Q || exit $?
timeout -k 10 900 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_c3_driver.log 2>&1 || exit $?
echo "c3 $(grep '^{' $O/bench_c3_driver.log | cut -c1-400)"
timeout -k 10 600 python3 -u bench.py --config c2 > $O/bench_c2.log 2>&1 || exit $?
echo "c2 $(grep '^{' $O/bench_c2.log | cut -c1-300)"
timeout -k 10 600 python3 -u bench.py --config c5 > $O/bench_c5.log 2>&1 || exit $?
echo "c5 $(grep '^{' $O/bench_c5.log | cut -c1-300)"
