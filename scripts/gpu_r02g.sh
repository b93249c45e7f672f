cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r02g
mkdir -p $O
MCMC_PROBE_MODES=0 timeout -k 10 300 python -u scripts/scan_probe.py c3 > $O/c3_default.log 2>&1 || exit $?
echo "default $(grep '^{' $O/c3_default.log | cut -c1-160)"
MCMC_HIP_LIB=mcmc_colorer_amd/variants/libmcmc_hip_bl.so MCMC_PROBE_MODES=0 timeout -k 10 300 python -u scripts/scan_probe.py c3 > $O/c3_bl.log 2>&1 || exit $?
echo "bufload $(grep '^{' $O/c3_bl.log | cut -c1-160)"
MCMC_PROBE_MODES=0 MCMC_PHASE_DUMP=$O/c3_early_sl1.phase timeout -k 10 300 python -u scripts/scan_probe.py c3 > $O/c3_phase.log 2>&1 || exit $?
python scripts/phase_summary.py $O/c3_early_sl1.phase | tail -4
for cfg in c3 c2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$cfg/trace -o run -- python3 bench.py --config $cfg --steps 20 --warmup 2 --no-cpu-baseline --no-convergence --no-refstruct --no-full-scan > $O/prof_${cfg}_trace.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_$cfg/pmc1 -o run -- python3 bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline --no-convergence --no-refstruct --no-full-scan > $O/prof_${cfg}_pmc1.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_$cfg/pmc2 -o run -- python3 bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline --no-convergence --no-refstruct --no-full-scan > $O/prof_${cfg}_pmc2.log 2>&1 || exit $?
  echo "prof $cfg ok"
done
find $O -name "*.csv" | head -20
