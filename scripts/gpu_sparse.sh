cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r02l; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_c3_full.py -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for d in 0 16 32 64; do
  MCMC_DRAIN_ROWS=$d MCMC_PROBE_MODES=0 timeout -k 10 300 python -u scripts/scan_probe.py c3 > $O/c3_d$d.log 2>&1 || exit $?
  echo "drain=$d $(grep '^{' $O/c3_d$d.log | cut -c1-150)"
done
MCMC_PROBE_MODES=0 timeout -k 10 300 python -u scripts/scan_probe.py c2 > $O/c2.log 2>&1 || exit $?
echo "c2 $(grep '^{' $O/c2.log | cut -c1-150)"
