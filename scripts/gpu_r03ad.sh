#!/bin/bash
# Walk LDS sized by nCol: wide parity suite; violator-heavy loop and converged C5 timeline,
# 1024 (in-tree) vs 2048 walk workgroups (variant library).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03ad}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_wide.py -m gpu -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for v in base wb2048 base wb2048; do
  if [ $v = base ]; then unset MCMC_HIP_LIB; else export MCMC_HIP_LIB=$PWD/mcmc_colorer_amd/variants/libmcmc_$v.so; fi
  timeout -k 10 300 python3 scripts/c5_viol_probe.py > $O/viol_$v.log 2>&1 || exit $?
  echo "$v: $(grep rep $O/viol_$v.log | tr '\n' ' ' | cut -c1-200)"
done
for v in base wb2048; do
  if [ $v = base ]; then unset MCMC_HIP_LIB; else export MCMC_HIP_LIB=$PWD/mcmc_colorer_amd/variants/libmcmc_$v.so; fi
  timeout -k 10 300 python3 -u bench.py --config c5 --steps 50 --warmup 20 --no-cpu-baseline --no-refstruct --no-convergence > $O/bench_$v.log 2>&1 || exit $?
  echo "$v: $(grep '^{' $O/bench_$v.log | tail -1 | cut -c150-200)"
done
