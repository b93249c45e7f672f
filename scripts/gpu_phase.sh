cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r02d
MCMC_PROBE_MODES=0 MCMC_PHASE_DUMP=gpurun_out/r02d/c3_early.phase timeout -k 10 300 python -u scripts/scan_probe.py c3 > gpurun_out/r02d/probe.log 2>&1
rc=$?; echo "probe rc=$rc"; grep '^{' gpurun_out/r02d/probe.log; [ $rc -ne 0 ] && exit $rc
python scripts/phase_summary.py gpurun_out/r02d/c3_early.phase
