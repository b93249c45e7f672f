#!/bin/bash
# r05: C5 persistent wide sweep, helper poll interval A/B (MCMC_WS_POLL: 0 spin, 1, 8)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r05l}; mkdir -p $O
for pl in ${POLLS:-1}; do
  MCMC_WS_POLL=$pl timeout -k 10 300 python -u bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline --no-refstruct --no-convergence > $O/c5_p$pl.log 2>&1 || { tail -5 $O/c5_p$pl.log; exit 1; }
  tail -1 $O/c5_p$pl.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.read()); w=d['wide_inc']['persistent']
print('poll=$pl c5', round(d['ms_per_step']*1e3,2), 'us', {k: round(v,1) for k,v in w['step_us_per_sweep'].items()}, [round(x,1) for x in w['probe_us_per_sweep']])"
done
