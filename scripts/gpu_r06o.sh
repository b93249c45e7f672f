cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r06o; mkdir -p $OUT
MCMC_DCM_BS=1024 timeout -k 5 90 python -u scripts/dcm_bs_probe.py > $OUT/bs1024.log 2>&1; rc=$?; echo "bs1024 rc=$rc"; tail -5 $OUT/bs1024.log
[ $rc -eq 0 ] || exit $rc
MCMC_DCM_BS=512 timeout -k 5 90 python -u scripts/dcm_bs_probe.py > $OUT/bs512.log 2>&1; rc=$?; echo "bs512 rc=$rc"; tail -5 $OUT/bs512.log
exit $rc
