#!/bin/bash
# r05 baseline at HEAD: C3 driver-shaped bench line, C5 default vs MCMC_WALK_LIGHT=0 (alternating).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 --no-refstruct --no-cpu-baseline --no-full-scan > $O/c3.log 2>&1 || exit $?
python3 - $O/c3.log <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('c3', round(d['ms_per_step']*1e3,2),'us', d['roofline']['kernel_ms'], d['convergence']['loop_ms'])
PY
for i in 1 2; do
  for wl in def 0; do
    if [ $wl = def ]; then unset MCMC_WALK_LIGHT; else export MCMC_WALK_LIGHT=0; fi
    timeout -k 10 300 python3 -u bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline --no-refstruct > $O/c5_${wl}_$i.log 2>&1 || exit $?
    tail -1 $O/c5_${wl}_$i.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('c5 wl=$wl $i', round(d['ms_per_step']*1e3,2), 'us; violators', round(d['violators']['ms_per_sweep']*1e3,1), 'us/sweep')"
  done
done
