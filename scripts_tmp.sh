cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29551 bench.py --config c2 --steps 20 --warmup 2 --backend gloo --same-device > gpurun_out/b_r2_c2.log 2>&1 || { echo "r2 c2 FAIL"; tail -20 gpurun_out/b_r2_c2.log; exit 1; }
tail -1 gpurun_out/b_r2_c2.log | cut -c1-700
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29552 bench.py --config c3 --steps 5 --warmup 1 --backend gloo --same-device > gpurun_out/b_r2_c3.log 2>&1 || { echo "r2 c3 FAIL"; tail -20 gpurun_out/b_r2_c3.log; exit 1; }
tail -1 gpurun_out/b_r2_c3.log | cut -c1-900
