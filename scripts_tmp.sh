cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 200 --warmup 10 > gpurun_out/bench.log 2>&1 || exit 1
tail -1 gpurun_out/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r01b/trace -o run -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/prof_trace.log 2>&1 || exit 2
grep sweep_kernel gpurun_out/prof_r01b/trace/run_kernel_stats.csv | cut -c1-200
