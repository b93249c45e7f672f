# One build-measure iteration on the GPU box: the parity tests of the single-GPU sweep, then the
# early-exit probe on C2 and C3 (and the C3 phase split). Usage: bash scripts/gpu_iter.sh TAG [pytest -k expr]
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1; mkdir -p $O
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "$K" > $O/pytest.log 2>&1
else
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
fi
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
MCMC_PROBE_MODES=0 timeout -k 10 300 python -u scripts/scan_probe.py c2 > $O/probe_c2.log 2>&1
rc=$?; echo "probe c2 rc=$rc"; grep '^{' $O/probe_c2.log | cut -c1-200
[ $rc -ne 0 ] && exit $rc
MCMC_PROBE_MODES=0 timeout -k 10 300 python -u scripts/scan_probe.py c3 > $O/probe_c3.log 2>&1
rc=$?; echo "probe c3 rc=$rc"; grep '^{' $O/probe_c3.log | cut -c1-200
[ $rc -ne 0 ] && exit $rc
if [ -n "${PHASE:-}" ]; then
  MCMC_PHASE_DUMP=$O/c3.phase MCMC_PROBE_MODES=0 timeout -k 10 300 python -u scripts/scan_probe.py c3 > $O/phase_run.log 2>&1 && python scripts/phase_summary.py $O/c3.phase | tail -4
fi
