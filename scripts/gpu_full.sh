#!/bin/bash
# Round check: GPU suite, smoke, default bench line, rocprof kernel trace + PMC passes (c3, c2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r02m}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u bench.py > $O/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench_default.log | cut -c1-600; [ $rc -ne 0 ] && exit $rc
for cfg in c3 c2; do
  A="--config $cfg --no-cpu-baseline --no-convergence --no-refstruct --no-full-scan"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$cfg/trace -o run -- python3 bench.py $A --steps 20 --warmup 2 > $O/prof_${cfg}_trace.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_$cfg/pmc1 -o run -- python3 bench.py $A --steps 5 --warmup 1 > $O/prof_${cfg}_pmc1.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_$cfg/pmc2 -o run -- python3 bench.py $A --steps 5 --warmup 1 > $O/prof_${cfg}_pmc2.log 2>&1 || exit $?
  echo "prof $cfg ok"
done
