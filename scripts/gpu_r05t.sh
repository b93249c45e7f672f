#!/bin/bash
# r05: persistent wide sweep tests, then C5 converged with the leader's heavy walks on / off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r05t}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_wide.py -k "persistent" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for lh in 0 1 0 1; do
  MCMC_WALK_TIE=$lh timeout -k 10 300 python -u bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline --no-refstruct > $O/c5_$lh.log 2>&1 || { tail -5 $O/c5_$lh.log; exit 1; }
  tail -1 $O/c5_$lh.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.read()); p=d['wide_inc']['persistent']
print('walk_tie=$lh c5', round(d['ms_per_step']*1e3,2), 'us', {k: round(v,2) for k,v in p['step_us_per_sweep'].items()}, 'leader_walks', p['leader_walks'], 'walk_phases', p['walk_phases'], 'viol_ms', round(d['violators']['ms_per_sweep'],4))"
done
