#!/bin/bash
# r06: the persistent wide sweep after a change: its -m gpu tests, the full-size C5 file, the C5 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r06ws}; mkdir -p $OUT
(while sleep 30; do date > $OUT/hb; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_wide.py tests/test_knobs.py tests/test_c5_full.py > $OUT/t.log 2>&1
rc=$?; tail -2 $OUT/t.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/t.log | head; exit $rc; }
timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --no-refstruct --no-convergence > $OUT/c5.json 2> $OUT/c5.err || exit 1
echo "c5: $(python3 -c "import json;d=json.loads(open('$OUT/c5.json').read().splitlines()[-1]);print(d['ms_per_step'], d['roofline']['kernel_ms'], d['wide_inc']['persistent']['step_us_per_sweep'], d['wide_inc']['changed_arcs_per_sweep'])")"
