#!/bin/bash
# r06: the persistent sweeps' helper poll interval against the leader's sweep time: the C5 bench
# (ws_kernel, MCMC_WS_POLL s_sleep(2) rounds) and the C3 bench (dc_multi_kernel, MCMC_DC_POLL
# s_sleep(4) rounds), 50 timed sweeps each, no CPU / refstruct / convergence legs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-poll}; mkdir -p $OUT
for p in 1 8 64; do
  MCMC_WS_POLL=$p timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --no-refstruct --no-convergence > $OUT/c5_poll$p.json 2> $OUT/c5_poll$p.err || exit $?
  echo "c5 poll $p: $(python3 -c "import json,sys;d=json.loads(open('$OUT/c5_poll$p.json').read().splitlines()[-1]);print(d['ms_per_step'], d['roofline']['kernel_ms'])")"
done
for p in 1 8 64; do
  MCMC_DC_POLL=$p timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-refstruct --no-convergence --no-full-scan > $OUT/c3_poll$p.json 2> $OUT/c3_poll$p.err || exit $?
  echo "c3 poll $p: $(python3 -c "import json,sys;d=json.loads(open('$OUT/c3_poll$p.json').read().splitlines()[-1]);print(d['ms_per_step'], d['roofline']['kernel_ms'])")"
done
