#!/bin/bash
# r05: candidates tested against the violator list in LDS -- persistent wide tests, C5 full size, C5 bench x2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r05x}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_wide.py tests/test_c5_full.py -k "persistent or c5" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config c5 --steps 50 --warmup 20 --no-cpu-baseline --no-refstruct --no-convergence > $O/c5_$i.log 2>&1 || { tail -5 $O/c5_$i.log; exit 1; }
  tail -1 $O/c5_$i.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.read()); p=d['wide_inc']['persistent']
print('c5', round(d['ms_per_step']*1e3,2), 'us', {k: round(v,2) for k,v in p['step_us_per_sweep'].items()})"
done
