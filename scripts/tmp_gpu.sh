#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_cli.py -m gpu -q -p no:cacheprovider > gpurun_out/pytest_cli.log 2>&1
rc=$?; echo "cli rc=$rc"; tail -3 gpurun_out/pytest_cli.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config c2 --semantics ref --steps 200 --warmup 20 > gpurun_out/bench_ref_c2.log 2>&1
rc=$?; echo "ref c2 rc=$rc"; tail -1 gpurun_out/bench_ref_c2.log | cut -c1-600; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --semantics ref --steps 20 --warmup 3 > gpurun_out/bench_ref_c3.log 2>&1
rc=$?; echo "ref c3 rc=$rc"; tail -1 gpurun_out/bench_ref_c3.log | cut -c1-600; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_prof.sh r01ref_c2 --config c2 --semantics ref --no-refstruct || exit $?
bash scripts/gpu_prof.sh r01ref_c3 --semantics ref --no-refstruct || exit $?
