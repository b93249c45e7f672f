#!/bin/bash
# r05: the persistent wide sweep -- wide tests (persistent first), then the C5 bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r05g}; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_wide.py -k "persistent" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/ws.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error" $O/ws.log | tail -20; tail -2 $O/ws.log
if [ $rc -ne 0 ]; then grep -n "assert\|Error" $O/ws.log | head -30; exit $rc; fi
timeout -k 10 600 python3 -u -m pytest tests/test_wide.py tests/test_knobs.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/wide.log 2>&1
rc=$?; tail -3 $O/wide.log
if [ $rc -ne 0 ]; then grep -n "assert\|Error\|FAIL" $O/wide.log | head -30; exit $rc; fi
timeout -k 10 300 python -u bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline --no-refstruct > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 1; }
tail -1 $O/c5.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('c5', round(d['ms_per_step']*1e3,2), 'us; violators', round(d['violators']['ms_per_sweep']*1e3,1), 'us/sweep', d['violators']['trajectory'][:4], 'loop', d['convergence']['loop_ms'])"
