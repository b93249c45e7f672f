#!/bin/bash
# Round-3 final check, part D: rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of the C3 and
# C5 benches at the bench's step counts, then the SQ/LDS counters of the C3 sweep.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r03final}
Q="--no-refstruct --no-convergence --no-full-scan --steps 50 --warmup 20"
bash scripts/gpu_prof.sh ${TAG}_c3 $Q || exit $?
bash scripts/gpu_prof.sh ${TAG}_c5 --config c5 $Q || exit $?
bash scripts/gpu_pmc_sq.sh ${TAG}_sq || exit $?
# A/B: 256 walk workgroups instead of 1024 (fewer workgroups to dispatch in the evaluation launch)
O=gpurun_out/${TAG}_wb; mkdir -p $O
export TMPDIR=/tmp
for v in base wb256; do
  if [ $v = base ]; then unset MCMC_HIP_LIB; else export MCMC_HIP_LIB=$PWD/mcmc_colorer_amd/variants/libmcmc_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t_$v -o run -- python3 bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline --no-refstruct --no-convergence > $O/bench_$v.log 2>&1 || exit $?
  echo "$v: $(grep '^{' $O/bench_$v.log | tail -1 | cut -c150-200)"
  python3 scripts/timeline.py $(find $O/t_$v -name "*kernel_trace.csv" | head -1) 8 | head -4
  timeout -k 10 300 python3 scripts/c5_viol_probe.py > $O/viol_$v.log 2>&1 || exit $?
  grep rep $O/viol_$v.log
done
unset MCMC_HIP_LIB
