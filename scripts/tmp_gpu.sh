cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in tiled tiled::::0; do
timeout -k 10 400 python bench.py --config c2 --steps 100 --warmup 5 --no-cpu-baseline --no-refstruct --variant $v > gpurun_out/b_c2v.log 2>&1 || { tail -5 gpurun_out/b_c2v.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/b_c2v.log').read().strip().splitlines()[-1]); print('c2 $v', '%.4f ms'%d['roofline']['kernel_ms'], '%.3e'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
done
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-refstruct > gpurun_out/b_c3v.log 2>&1 && python -c "import json; d=json.loads(open('gpurun_out/b_c3v.log').read().strip().splitlines()[-1]); print('c3', '%.3f ms'%d['roofline']['kernel_ms'], '%.3e'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
