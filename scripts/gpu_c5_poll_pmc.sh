#!/bin/bash
# r06: C5 ws_kernel FETCH_SIZE / timing against the helpers' idle poll interval (MCMC_WS_POLL_IDLE):
# does the PMC read traffic come from the polls or from the sweep's random gathers?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06c5p}; mkdir -p $OUT
for p in 0 16 1000; do
  MCMC_WS_POLL_IDLE=$p timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/p$p -o run -- python3 bench.py --config c5 --no-cpu-baseline --no-refstruct --no-convergence > $OUT/p$p.log 2>&1 || exit $?
  echo "idle $p: $(python3 -c "
import csv
v=[float(r['Counter_Value']) for r in csv.DictReader(open('$OUT/p$p/run_counter_collection.csv')) if r['Counter_Name']=='FETCH_SIZE' and 'ws_kernel' in r['Kernel_Name']]
print([round(x) for x in v])") $(grep -o '\"ms_per_step\": [0-9.e-]*' $OUT/p$p.log | head -1)"
done
