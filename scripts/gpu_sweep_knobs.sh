cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r02e
for sl in 0 1 2 3; do
  MCMC_PROBE_MODES=0 MCMC_SUB_LOG2=$sl timeout -k 10 300 python -u scripts/scan_probe.py c3 > gpurun_out/r02e/c3_sl$sl.log 2>&1 || exit $?
  echo "sl=$sl $(grep '^{' gpurun_out/r02e/c3_sl$sl.log | cut -c1-200)"
  MCMC_PROBE_MODES=0 MCMC_SUB_LOG2=$sl timeout -k 10 300 python -u scripts/scan_probe.py c2 > gpurun_out/r02e/c2_sl$sl.log 2>&1 || exit $?
  echo "sl=$sl $(grep '^{' gpurun_out/r02e/c2_sl$sl.log | cut -c1-200)"
done
