#!/bin/bash
# r05: tie-binade walk on by default -- every wide test, the wide knobs, the multi-GPU wide tests,
# the full-size C5 file and the C3 default-nCol test
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r05u}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_wide.py tests/test_knobs.py tests/test_multi.py tests/test_c5_full.py "tests/test_c3_full.py::test_c3_default_ncol_maxdeg_sampled_rows" > $O/t.log 2>&1; rc=$?
tail -3 $O/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline --no-refstruct > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 1; }
tail -1 $O/c5.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.read()); p=d['wide_inc']['persistent']
print('c5', round(d['ms_per_step']*1e3,2), 'us', {k: round(v,2) for k,v in p['step_us_per_sweep'].items()}, 'viol_ms', round(d['violators']['ms_per_sweep'],4))"
