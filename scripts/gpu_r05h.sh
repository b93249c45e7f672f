#!/bin/bash
# r05: C5 bench with the persistent wide sweep's per-step times, and with it off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r05h}; mkdir -p $O
for ws in 1 0; do
  MCMC_WIDE_SOLO=$ws timeout -k 10 300 python -u bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline --no-refstruct > $O/c5_ws$ws.log 2>&1 || { tail -5 $O/c5_ws$ws.log; exit 1; }
  tail -1 $O/c5_ws$ws.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.read()); w=d.get('wide_inc',{})
print('ws=$ws c5', round(d['ms_per_step']*1e3,2), 'us; violators', round(d['violators']['ms_per_sweep']*1e3,1), 'us/sweep', d['violators']['trajectory'][:4], 'loop', round(d['convergence']['loop_ms'],3))
print('   persistent', json.dumps(w.get('persistent'))[:1300])"
done
