#!/bin/bash
# r06: the C3 bench line with and without the solo sweep's candidate prefetch (MCMC_DC_PF), alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r06pfab}; mkdir -p $OUT
for r in 1 2 3; do for pf in 1 0; do
  MCMC_DC_PF=$pf timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-refstruct --no-full-scan > $OUT/c3_pf${pf}_$r.json 2>/dev/null || exit 1
  echo "pf $pf run $r: $(python3 -c "import json;d=json.loads(open('$OUT/c3_pf${pf}_$r.json').read().splitlines()[-1]);print(d['ms_per_step'], d['roofline']['kernel_ms'], d['convergence']['loop_ms'])")"
done; done
