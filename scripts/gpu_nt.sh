cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r02h; mkdir -p $O
for v in default nt; do
  L=""; [ $v = nt ] && L=mcmc_colorer_amd/variants/libmcmc_hip_nt.so
  MCMC_HIP_LIB=${L:-mcmc_colorer_amd/libmcmc_hip.so} MCMC_PROBE_MODES=0 timeout -k 10 300 python -u scripts/scan_probe.py c3 > $O/c3_$v.log 2>&1 || exit $?
  echo "$v $(grep '^{' $O/c3_$v.log | cut -c1-120)"
  MCMC_HIP_LIB=${L:-mcmc_colorer_amd/libmcmc_hip.so} MCMC_PROBE_MODES=1 timeout -k 10 300 python -u scripts/scan_probe.py c3 > $O/c3_full_$v.log 2>&1 || exit $?
  echo "$v full $(grep '^{' $O/c3_full_$v.log | cut -c1-120)"
done
