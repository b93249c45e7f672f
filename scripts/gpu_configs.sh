cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/${1:-r02n}; mkdir -p $O
timeout -k 10 600 python -u bench.py --config c2 --steps 200 --warmup 10 > $O/bench_c2.log 2>&1 || exit $?
echo "c2 $(tail -1 $O/bench_c2.log | cut -c1-300)"
timeout -k 10 600 python -u bench.py --config c5 --steps 50 --warmup 5 > $O/bench_c5.log 2>&1 || exit $?
echo "c5 $(tail -1 $O/bench_c5.log | cut -c1-300)"
timeout -k 10 300 python -u bench.py --force-dist --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-refstruct > $O/bench_c3_dist1.log 2>&1 || exit $?
echo "c3 dist1 $(tail -1 $O/bench_c3_dist1.log | cut -c1-300)"
timeout -k 10 300 python -u bench.py --force-dist --config c2 --steps 200 --warmup 10 --no-cpu-baseline --no-refstruct > $O/bench_c2_dist1.log 2>&1 || exit $?
echo "c2 dist1 $(tail -1 $O/bench_c2_dist1.log | cut -c1-300)"
MCMC_PROBE_MODES=0 MCMC_PHASE_DUMP=$O/c3.phase timeout -k 10 300 python -u scripts/scan_probe.py c3 > $O/c3_phase.log 2>&1 || exit $?
python scripts/phase_summary.py $O/c3.phase | tail -4
