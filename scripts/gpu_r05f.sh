#!/bin/bash
# r05: C5 A/B -- base (in-tree lib) vs variants/libmcmc_<v>.so and MCMC_WALK_LIGHT=0, then a kernel
# trace of base. Usage: scripts/gpu_r05f.sh TAG "v1 v2"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05f}; mkdir -p $O
B="bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline --no-refstruct"
show() { tail -1 $1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$2', round(d['ms_per_step']*1e3,2), 'us; violators', round(d['violators']['ms_per_sweep']*1e3,1), 'us/sweep', d['violators']['trajectory'][:4])"; }
for i in 1 2; do
  for v in base $2 light0; do
    unset MCMC_HIP_LIB MCMC_WALK_LIGHT
    [ $v = light0 ] && export MCMC_WALK_LIGHT=0
    [ $v != base ] && [ $v != light0 ] && export MCMC_HIP_LIB=$PWD/variants/libmcmc_$v.so
    timeout -k 10 300 python -u $B > $O/${v}_$i.log 2>&1 || { tail -5 $O/${v}_$i.log; exit 1; }
    show $O/${v}_$i.log $v$i
  done
done
unset MCMC_HIP_LIB MCMC_WALK_LIGHT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --config c5 --steps 30 --warmup 3 --no-cpu-baseline --no-refstruct --no-convergence > $O/trace.log 2>&1
rc=$?; echo "trace rc=$rc"
python3 scripts/trace_avg.py $O/trace/run_kernel_trace.csv 2>/dev/null | tail -8 || find $O/trace -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1-6 | head
exit $rc
