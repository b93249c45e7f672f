#!/bin/bash
# r05: hybrid path choice (persistent wide sweep only near convergence): ws tests, C5 violator loop, C5 bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r05m}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_wide.py tests/test_multi.py -k "persistent or world1 or matches_oracle" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -3 $O/t.log
timeout -k 10 200 python -u scripts/ws_viol.py > $O/viol.log 2>&1 || { tail -5 $O/viol.log; exit 1; }
cat $O/viol.log
timeout -k 10 300 python -u bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline --no-refstruct > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 1; }
tail -1 $O/c5.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.read()); h=d['headline']
print('c5', round(d['ms_per_step']*1e3,2), 'us/sweep converged;', {k: round(v['ms_per_sweep'],4) for k,v in h.items() if isinstance(v, dict)})"
