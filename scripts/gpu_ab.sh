# A/B of two library builds on the C3 (and C2) probe, alternating: A = in-tree lib, B = $B_LIB.
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1; mkdir -p $O
for i in 1 2; do
  for v in A B; do
    if [ $v = B ]; then export MCMC_HIP_LIB=$B_LIB; else unset MCMC_HIP_LIB; fi
    MCMC_PROBE_MODES=0 timeout -k 10 300 python -u scripts/scan_probe.py ${CFG:-c3} > $O/${v}_$i.log 2>&1 || exit $?
    echo "$v$i $(grep '^{' $O/${v}_$i.log | cut -c40-120)"
  done
done
