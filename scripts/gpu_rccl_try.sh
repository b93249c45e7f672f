cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03a
timeout -k 10 400 python -u -m pytest tests/test_rccl_world.py -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread -k "er-rows-p2p and 2" > gpurun_out/r03a/rccl.log 2>&1
rc=$?; echo rc=$rc; tail -30 gpurun_out/r03a/rccl.log
