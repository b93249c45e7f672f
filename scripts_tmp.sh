cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/b_default.log 2>&1 || { echo "bench FAIL"; tail -5 gpurun_out/b_default.log; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/b_default.log').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['refstruct']['speedup'], d['cpu_baseline']['value'])"
timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline > gpurun_out/b_c2.log 2>&1 || { echo "c2 FAIL"; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/b_c2.log').read().strip().splitlines()[-1])
print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['refstruct']['speedup'])"
bash scripts_gpu_prof.sh r01_c3b --config c3 --no-refstruct && bash scripts_gpu_prof.sh r01_c2b --config c2 --no-refstruct
