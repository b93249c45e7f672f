cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r02c
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_multi.py tests/test_gpu_refmode.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r02c/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r02c/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/scan_probe.py c2 > gpurun_out/r02c/probe_c2.log 2>&1
rc=$?; echo "probe c2 rc=$rc"; grep '^{' gpurun_out/r02c/probe_c2.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/scan_probe.py c3 > gpurun_out/r02c/probe_c3.log 2>&1
rc=$?; echo "probe c3 rc=$rc"; grep '^{' gpurun_out/r02c/probe_c3.log
exit $rc
