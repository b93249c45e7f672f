#!/bin/bash
# Device tie-binade scan (MCMC_WALK_TIE=1) vs the default: wide parity both ways, walk timings, violator loop.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03ak}; mkdir -p $O
MCMC_WALK_TIE=1 timeout -k 10 600 python -u -m pytest tests/test_wide.py tests/test_c5_full.py -m gpu -x -q -p no:cacheprovider \
    --timeout 500 --timeout-method thread > $O/pytest_tie.log 2>&1
rc=$?; echo "pytest (tie scan) rc=$rc"; tail -3 $O/pytest_tie.log; [ $rc -ne 0 ] && exit $rc
MCMC_WALK_TIE=1 timeout -k 10 300 python3 -u scripts/walk_probe.py $O/w.bin > $O/walk_tie.log 2>&1 || exit $?
grep -v amdgpu.ids $O/walk_tie.log; rm -f $O/w.bin
for i in 1 2; do
  MCMC_WALK_TIE=1 timeout -k 10 300 python3 scripts/c5_viol_probe.py > $O/viol_tie_$i.log 2>&1 || exit $?
  echo "tie: $(grep rep $O/viol_tie_$i.log | tr '\n' ' ' | cut -c1-220)"
  timeout -k 10 300 python3 scripts/c5_viol_probe.py > $O/viol_def_$i.log 2>&1 || exit $?
  echo "def: $(grep rep $O/viol_def_$i.log | tr '\n' ' ' | cut -c1-220)"
done
timeout -k 10 600 python -u -m pytest tests/test_wide.py -m gpu -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread > $O/pytest_def.log 2>&1
rc=$?; echo "pytest (default) rc=$rc"; tail -2 $O/pytest_def.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --config c5 > $O/bench_c5.log 2>&1 || exit $?
grep '^{' $O/bench_c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', d['ms_per_step'], d['value'], d.get('violators'))"
