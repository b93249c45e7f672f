#!/bin/bash
# Fast wide commit, wave-aggregated violator flags, split hub deltas: wide parity suite, full-size C5
# check, C5 timelines (converged, violator-heavy), C5 bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03w}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_wide.py -m gpu -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_c5_full.py -m gpu -x -v -s -p no:cacheprovider \
    --timeout 600 --timeout-method thread > $O/pytest_c5_full.log 2>&1
rc=$?; echo "c5 full rc=$rc"; tail -6 $O/pytest_c5_full.log; [ $rc -ne 0 ] && exit $rc
Q="--config c5 --steps 20 --warmup 5 --no-cpu-baseline --no-refstruct --no-convergence"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t1 -o run -- python3 bench.py $Q > $O/bench_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
f=$(find $O/t1 -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py $f 8 | head -4
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tv -o run -- python3 scripts/c5_viol_probe.py > $O/viol.log 2>&1
rc=$?; echo "viol rc=$rc"; grep rep $O/viol.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --config c5 --no-refstruct --no-cpu-baseline > $O/bench_c5.log 2>&1
rc=$?; echo "bench c5 rc=$rc"; [ $rc -ne 0 ] && exit $rc
grep '^{' $O/bench_c5.log | tail -1 > $O/bench_c5.json
python3 - $O/bench_c5.json <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
print(d["ms_per_step"], d.get("violators"), d.get("headline",{}).get("reference_loop"), {k: v for k, v in (d.get("wide_inc") or {}).items() if k != "note"})
PY
