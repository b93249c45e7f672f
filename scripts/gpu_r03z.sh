#!/bin/bash
# Wide parity + C5 timeline (commit: draw coefficients only for the events present); C2 phase dump.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03z}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_wide.py -m gpu -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
Q="--config c5 --steps 20 --warmup 5 --no-cpu-baseline --no-refstruct --no-convergence"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t1 -o run -- python3 bench.py $Q > $O/bench_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
f=$(find $O/t1 -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py $f 8 | head -4
MCMC_PROBE_MODES=0 MCMC_PHASE_DUMP=$O/c2.phase timeout -k 10 300 python -u scripts/scan_probe.py c2 > $O/c2probe.log 2>&1
rc=$?; echo "c2 phase rc=$rc"; grep '^{' $O/c2probe.log | cut -c1-120; [ $rc -ne 0 ] && exit $rc
python3 scripts/phase_summary.py $O/c2.phase
for v in default nosplit; do
  if [ $v = nosplit ]; then export MCMC_SPLIT_ARCS=1048576; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tv_$v -o run -- python3 scripts/c5_viol_probe.py > $O/viol_$v.log 2>&1
  rc=$?; echo "viol $v rc=$rc"; grep rep $O/viol_$v.log; [ $rc -ne 0 ] && exit $rc
done
unset MCMC_SPLIT_ARCS
exit 0
