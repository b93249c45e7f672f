cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r02i; mkdir -p $O
for k in 1 2 3 4 5 6 8; do
  MCMC_DEBUG_MAX_PAIRS=$k MCMC_PROBE_MODES=0 timeout -k 10 300 python -u scripts/scan_probe.py c3 > $O/c3_k$k.log 2>&1 || exit $?
  echo "k=$k $(grep '^{' $O/c3_k$k.log | cut -c1-190)"
done
