cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/b_default.log 2>&1 || { echo "bench FAIL"; tail -5 gpurun_out/b_default.log; exit 1; }
tail -1 gpurun_out/b_default.log | cut -c1-600
bash scripts_gpu_prof.sh r01_tiled
