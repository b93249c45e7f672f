#!/bin/bash
# GreedyFF parity (restatement, CLI files) then the whole GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_greedyff.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gff_tests.log 2>&1
rc=$?; echo "gff tests rc=$rc"; tail -12 gpurun_out/gff_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
exit $rc
