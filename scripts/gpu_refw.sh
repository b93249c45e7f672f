# REF-wide check: the reference-semantics parity tests, then a kernel-trace profile of the C5
# stand-in with --semantics ref. Usage: bash scripts/gpu_refw.sh TAG
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_refmode.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "${K:-wide}" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --config c5 --semantics ref --steps 10 --warmup 2 --no-cpu-baseline --no-refstruct --no-convergence > $O/bench.log 2>&1
rc=$?; grep -h refw $O/trace/run_kernel_stats.csv | cut -c1-130; tail -1 $O/bench.log | cut -c1-300
exit $rc
