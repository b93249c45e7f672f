cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
run() { name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/b_$name.log 2>&1 || { echo "FAIL $name"; tail -5 gpurun_out/b_$name.log; exit 1; }; python -c "
import json,sys
d=json.loads(open('gpurun_out/b_$name.log').read().strip().splitlines()[-1]); print('$name', '%.3e'%d['value'], 'step %.4f ms'%d['ms_per_step'], 'kern %.4f ms'%d['roofline']['kernel_ms'], 'frac %.3f'%d['roofline']['frac'], d['config']['workload'])"; }
run default python bench.py --steps 100 --warmup 5 --no-cpu-baseline
run dist1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --steps 100 --warmup 5 --force-dist
run dist1_n8e5 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29534 bench.py --steps 50 --warmup 5 --force-dist --n 800000 --prob 0.00125
