# C5 A/B: bench --config c5 (converged timed sweeps + the violators record) for the in-tree library
# and variants/libmcmc_$v.so. Usage: bash scripts/gpu_c5ab.sh TAG "w512 w1024"
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1; mkdir -p $O
for v in base $2; do
  if [ $v = base ]; then unset MCMC_HIP_LIB; else export MCMC_HIP_LIB=$PWD/variants/libmcmc_$v.so; fi
  timeout -k 10 300 python -u bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --no-refstruct > $O/c5_$v.log 2>&1 || exit $?
  tail -1 $O/c5_$v.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$v', round(d['ms_per_step'],4), 'viol', round(d['violators']['ms_per_sweep'],4), d['violators']['trajectory'])"
done
