#!/bin/bash
# r05 (diagnostic): leader heavy walks with probes -- gather vs mask walk per heavy violator
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r05v}; mkdir -p $O
MCMC_WS_LEAD_HEAVY=65536 timeout -k 10 300 python -u bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline --no-refstruct --no-convergence > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 1; }
tail -1 $O/c5.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.read()); p=d['wide_inc']['persistent']
print('c5', round(d['ms_per_step']*1e3,2), 'us', {k: round(v,2) for k,v in p['step_us_per_sweep'].items()}, [round(x,2) for x in p['probe_us_per_sweep']], p['leader_walks'])"
