cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x -k "tiled or gather or lockstep or golden or unsorted or grid" > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
ph() { name=$1; shift; MCMC_PHASE_DUMP=gpurun_out/ph_$name.bin timeout -k 10 300 python bench.py --warmup 3 --no-cpu-baseline "$@" > gpurun_out/b_$name.log 2>&1 || { tail -5 gpurun_out/b_$name.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/b_$name.log').read().strip().splitlines()[-1]); print('$name', '%.4f ms'%d['roofline']['kernel_ms'], '%.3e'%d['value'], 'frac %.3f'%d['roofline']['frac'], d['roofline']['layout']['grp_rows'], d['roofline']['layout']['sub_log2'])"
python scripts_phase.py gpurun_out/ph_$name.bin | tail -4; }
ph c2 --steps 50
ph c2_stream --steps 50 --variant tiled::::1
ph n8e5 --steps 20 --n 800000 --prob 0.00125
ph n8e5_s1 --steps 20 --n 800000 --prob 0.00125 --variant tiled:16:1
ph n8e5_s3 --steps 20 --n 800000 --prob 0.00125 --variant tiled:16:3
