cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x -k "er_fast" > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-refstruct > gpurun_out/b_c3.log 2>&1; rc=$?
echo "c3 rc=$rc"; tail -3 gpurun_out/b_c3.log | cut -c1-1500
