cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x -k "tiled or gather or lockstep or golden or unsorted or er_fast or grid" > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
ph() { name=$1; shift; MCMC_PHASE_DUMP=gpurun_out/ph_$name.bin timeout -k 10 400 python bench.py --warmup 2 --no-cpu-baseline --no-refstruct "$@" > gpurun_out/b_$name.log 2>&1 || { tail -5 gpurun_out/b_$name.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/b_$name.log').read().strip().splitlines()[-1]); print('$name', '%.4f ms'%d['roofline']['kernel_ms'], '%.3e'%d['value'], 'frac %.3f'%d['roofline']['frac'], 'R', d['roofline']['layout']['grp_rows'])"
python scripts_phase.py gpurun_out/ph_$name.bin | tail -7; }
ph c3 --steps 10
ph c2 --steps 50 --config c2
ph c2s --steps 50 --config c2 --variant tiled::::1
