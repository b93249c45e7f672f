#!/bin/bash
# C5 (configs[4] stand-in): wide-sweep + R-MAT parity, the whole GPU suite, the c5 bench line and a
# rocprofv3 kernel trace of it. Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-c5}
timeout -k 10 400 python -u -m pytest tests/test_wide.py tests/test_rmat.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c5_tests.log 2>&1
rc=$?; echo "wide tests rc=$rc"; tail -25 gpurun_out/c5_tests.log; [ $rc -ne 0 ] && exit $rc
if [ -z "$SKIP_SUITE" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "suite rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 600 python -u bench.py --config c5 --steps 20 --warmup 3 "$@" > gpurun_out/bench_c5.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_c5.log | cut -c1-3000; [ $rc -ne 0 ] && exit $rc
if [ -n "$DIST" ]; then   # the partitioned driver: world 1 over RCCL, world 2 on one GPU over gloo
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --config c5 --steps 10 --warmup 2 --no-cpu-baseline --no-refstruct > gpurun_out/bench_c5_d1.log 2>&1
  rc=$?; echo "dist1 rc=$rc"; tail -1 gpurun_out/bench_c5_d1.log | cut -c1-600; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --config c5 --steps 5 --warmup 1 --backend gloo --same-device --no-cpu-baseline --no-refstruct > gpurun_out/bench_c5_d2.log 2>&1
  rc=$?; echo "dist2 rc=$rc"; tail -1 gpurun_out/bench_c5_d2.log | cut -c1-600; [ $rc -ne 0 ] && exit $rc
fi
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --config c5 --steps 20 --warmup 2 --no-cpu-baseline --no-refstruct "$@" > $OUT/bench_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -1 $OUT/bench_trace.log | cut -c1-400
find $OUT -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200 | head -14
exit $rc
