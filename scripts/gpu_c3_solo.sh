#!/bin/bash
# r06: C3 bench (no CPU / refstruct / full-scan legs) with the leader's per-step stamps
# (MCMC_SOLO_TRACE), summarised by scripts/solo_trace.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r06solo}; mkdir -p $OUT
MCMC_SOLO_TRACE=$OUT/solo.bin timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-refstruct --no-full-scan > $OUT/c3.json 2> $OUT/c3.err || exit 1
echo "c3: $(python3 -c "import json;d=json.loads(open('$OUT/c3.json').read().splitlines()[-1]);print(d['ms_per_step'], d['roofline']['kernel_ms'], d['convergence']['loop_ms'], d['convergence']['rebuild_ms'])")"
python3 scripts/solo_trace.py $OUT/solo.bin
