#!/bin/bash
# C5 A/B of library builds (in-tree lib = base, variants/libmcmc_<v>.so): the bench's converged sweep
# and its violator-heavy record, alternating twice. Usage: scripts/gpu_c5ab.sh TAG "v1 v2 ..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$1; mkdir -p $O
for i in 1 2; do
  for v in base $2; do
    if [ $v = base ]; then unset MCMC_HIP_LIB; else export MCMC_HIP_LIB=$PWD/variants/libmcmc_$v.so; fi
    timeout -k 10 300 python -u bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline --no-refstruct > $O/${v}_$i.log 2>&1 || exit $?
    tail -1 $O/${v}_$i.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$v$i', round(d['ms_per_step']*1e3,2), 'us; violators', round(d['violators']['ms_per_sweep']*1e3,1), 'us/sweep', d['violators']['trajectory'][:5])"
  done
done
