#!/bin/bash
# r05: the -m gpu suite without the full-size files (those: gpu_r05q.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r05p}; mkdir -p $O
timeout -k 10 200 python -u scripts/rt_exit_probe.py > $O/rt.log 2>&1; cat $O/rt.log
timeout -k 10 1000 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests \
  --ignore=tests/test_c3_full.py --ignore=tests/test_c4_full.py --ignore=tests/test_c5_full.py \
  --ignore=tests/test_rccl_world.py > $O/t.log 2>&1; rc=$?
tail -5 $O/t.log; exit $rc
