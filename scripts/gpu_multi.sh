cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r02b
timeout -k 10 600 python -u -m pytest tests/test_multi.py tests/test_gpu_parity.py tests/test_wide.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r02b/pytest_multi.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r02b/pytest_multi.log | tail -15
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --force-dist --config c2 --steps 200 --warmup 10 > gpurun_out/r02b/bench_c2_dist1.log 2>&1
rc=$?; echo "bench c2 dist1 rc=$rc"; tail -c 1500 gpurun_out/r02b/bench_c2_dist1.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --force-dist --config c3 --steps 20 --warmup 3 > gpurun_out/r02b/bench_c3_dist1.log 2>&1
rc=$?; echo "bench c3 dist1 rc=$rc"; tail -c 1500 gpurun_out/r02b/bench_c3_dist1.log
exit $rc
