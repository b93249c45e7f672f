cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r02f
for sl in 0 1 2; do
  MCMC_HIP_LIB=mcmc_colorer_amd/variants/libmcmc_hip_u8.so MCMC_PROBE_MODES=0 MCMC_SUB_LOG2=$sl timeout -k 10 300 python -u scripts/scan_probe.py c3 > gpurun_out/r02f/c3_u8_sl$sl.log 2>&1 || exit $?
  echo "u8 sl=$sl $(grep '^{' gpurun_out/r02f/c3_u8_sl$sl.log | cut -c1-160)"
done
for sl in 0 1; do
  MCMC_HIP_LIB=mcmc_colorer_amd/variants/libmcmc_hip_u8.so MCMC_PROBE_MODES=0 MCMC_SUB_LOG2=$sl timeout -k 10 300 python -u scripts/scan_probe.py c2 > gpurun_out/r02f/c2_u8_sl$sl.log 2>&1 || exit $?
  echo "u8 sl=$sl $(grep '^{' gpurun_out/r02f/c2_u8_sl$sl.log | cut -c1-160)"
done
