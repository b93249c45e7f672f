#!/bin/bash
# r03 probe: RCCL world 2 over the socket transport on one GPU (NCCL_HOSTID per rank), and the
# world-1 native driver's per-step overhead under a kernel trace (C2 and C3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03probe}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_rccl_world.py -m gpu -x -v -p no:cacheprovider --timeout 240 \
    --timeout-method thread -k "er-rows-p2p and 2" > $OUT/rccl.log 2>&1
echo "rccl rc=$?"; tail -5 $OUT/rccl.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c2d -o c2d -- python3 bench.py --config c2 --force-dist \
    --steps 40 --warmup 5 --no-cpu-baseline --no-refstruct > $OUT/c2d.log 2>&1
echo "c2 dist rc=$?"; tail -1 $OUT/c2d.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/c3d -o c3d -- python3 bench.py --config c3 --force-dist \
    --steps 20 --warmup 3 --no-cpu-baseline --no-refstruct > $OUT/c3d.log 2>&1
echo "c3 dist rc=$?"; tail -1 $OUT/c3d.log | cut -c1-400
find $OUT -name "*stats*.csv" | head
