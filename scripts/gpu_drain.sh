cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r02k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_wide.py tests/test_multi.py -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for d in 0 32 64 96 128; do
  MCMC_DRAIN_ROWS=$d MCMC_PROBE_MODES=0 timeout -k 10 300 python -u scripts/scan_probe.py c3 > $O/c3_d$d.log 2>&1 || exit $?
  echo "drain=$d $(grep '^{' $O/c3_d$d.log | cut -c1-150)"
done
