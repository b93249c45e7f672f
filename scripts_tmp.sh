cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python bench.py --config c3 > gpurun_out/b_c3_full.log 2>&1 || { echo "c3 full FAIL"; tail -5 gpurun_out/b_c3_full.log; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/b_c3_full.log').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['config']['graph_gen_s']); print(d['refstruct']); print(d['cpu_baseline'])"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --config c3 --steps 10 --warmup 2 --force-dist > gpurun_out/b_c3_dist1.log 2>&1 || { echo "c3 dist FAIL"; tail -5 gpurun_out/b_c3_dist1.log; exit 1; }
tail -1 gpurun_out/b_c3_dist1.log | cut -c1-400
bash scripts_gpu_prof.sh r01_c3 --config c3
