#!/bin/bash
# Dense-list incremental wide sweep + scalar skip-ahead: parity suites (wide, tiled, partitioned),
# C5 kernel timeline, C5 bench line, short C2 / C3 lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03u}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_wide.py tests/test_gpu_parity.py tests/test_multi.py -m gpu -x -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
Q="--config c5 --steps 20 --warmup 5 --no-cpu-baseline --no-refstruct --no-convergence"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t1 -o run -- python3 bench.py $Q > $O/bench_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
f=$(find $O/t1 -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py $f 8 | head -4
python3 scripts/trace_avg.py $f 40
timeout -k 10 600 python -u bench.py --config c5 --no-refstruct --no-cpu-baseline > $O/bench_c5.log 2>&1
rc=$?; echo "bench c5 rc=$rc"; [ $rc -ne 0 ] && exit $rc
grep '^{' $O/bench_c5.log | tail -1 > $O/bench_c5.json
python3 - $O/bench_c5.json <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
print(d["ms_per_step"], d.get("violators"), d.get("headline",{}).get("reference_loop"), {k: v for k, v in (d.get("wide_inc") or {}).items() if k != "note"})
PY
Q="--no-refstruct --no-convergence --no-cpu-baseline --no-full-scan"
timeout -k 10 300 python -u bench.py --config c2 $Q > $O/bench_c2.log 2>&1
rc=$?; echo "bench c2 rc=$rc"; tail -1 $O/bench_c2.log | cut -c1-260; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py $Q > $O/bench_c3.log 2>&1
rc=$?; echo "bench c3 rc=$rc"; tail -1 $O/bench_c3.log | cut -c1-260
exit $rc
