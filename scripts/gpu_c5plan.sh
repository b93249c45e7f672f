#!/bin/bash
# C5 tile-scan piece plans: the XCD-aware plan (default) vs the XCD-blind LPT plan -- bench line,
# kernel stats and tscan FETCH_SIZE of each, then the wide parity tests. Usage: scripts/gpu_c5plan.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-c5plan}; mkdir -p $O
B="bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline --no-refstruct --no-convergence"
for plan in xcd lpt xcd; do
  export MCMC_TSCAN_PLAN=$plan
  timeout -k 10 300 python -u $B > $O/bench_$plan.log 2>&1 || exit $?
  echo "$plan $(tail -1 $O/bench_$plan.log | cut -c100-200)"
done
for plan in xcd lpt; do
  export MCMC_TSCAN_PLAN=$plan
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$plan -o run -- python3 bench.py --config c5 --steps 20 --warmup 2 --no-cpu-baseline --no-refstruct --no-convergence > $O/trace_$plan.log 2>&1 || exit $?
  grep -h "wide_\|commit" $O/trace_$plan/run_kernel_stats.csv | cut -d, -f1-4 | sed "s/^/$plan /"
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$plan -o run -- python3 bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline --no-refstruct --no-convergence > $O/pmc_$plan.log 2>&1 || exit $?
  python3 - $O/pmc_$plan/run_counter_collection.csv $plan <<'PY'
import csv, sys
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(sys.argv[1])) if r["Counter_Name"] == "FETCH_SIZE" and "wide_tscan" in r["Kernel_Name"]]
print(sys.argv[2], "tscan FETCH_SIZE KiB (raw, last 4):", [round(x) for x in v[-4:]])
PY
done
unset MCMC_TSCAN_PLAN
timeout -k 10 600 python -u -m pytest tests/test_wide.py tests/test_multi.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_wide.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_wide.log
exit $rc
