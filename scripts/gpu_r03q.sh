#!/bin/bash
# Slot-listed incremental wide sweep: wide parity suite, C5 kernel timeline (inc on/off), C5 bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03q}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_wide.py tests/test_rmat.py -m gpu -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
Q="--config c5 --steps 20 --warmup 5 --no-cpu-baseline --no-refstruct --no-convergence"
MCMC_WIDE_INC=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t1 -o run -- python3 bench.py $Q > $O/bench_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
f=$(find $O/t1 -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py $f 16
python3 scripts/trace_avg.py $f 40
timeout -k 10 600 python -u bench.py --config c5 --no-refstruct --no-cpu-baseline > $O/bench_c5.log 2>&1
rc=$?; echo "bench c5 rc=$rc"
python - $O/bench_c5.log <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["ms_per_step"], d.get("violators"), d.get("headline",{}).get("reference_loop"), d.get("wide_inc"))
PY
