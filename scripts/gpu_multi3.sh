#!/bin/bash
# r03: the partitioned path -- loopback tests (delta / p2p / overflow / tail cut), the CLI on
# --gpus N --loopback, RCCL multi-process worlds on one GPU (socket transport via NCCL_HOSTID).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03multi}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_multi.py tests/test_cli.py -m gpu -x -v -p no:cacheprovider \
    --timeout 240 --timeout-method thread > $OUT/pytest_multi.log 2>&1
rc=$?; echo "multi rc=$rc"; tail -5 $OUT/pytest_multi.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_rccl_world.py -m gpu -x -v -p no:cacheprovider \
    --timeout 280 --timeout-method thread > $OUT/pytest_rccl.log 2>&1
rc=$?; echo "rccl rc=$rc"; tail -5 $OUT/pytest_rccl.log
exit $rc
