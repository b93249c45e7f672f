#!/bin/bash
# C5 incremental sweep: kernel timelines at hub thresholds 256 / 2048 / 65536.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03s}; mkdir -p $O
Q="--config c5 --steps 20 --warmup 5 --no-cpu-baseline --no-refstruct --no-convergence"
for h in 256 2048 65536; do
  MCMC_WIDE_INC_HUB=$h timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/h$h -o run -- python3 bench.py $Q > $O/bench_h$h.log 2>&1
  rc=$?; echo "hub $h rc=$rc"; [ $rc -ne 0 ] && exit $rc
  f=$(find $O/h$h -name "*kernel_trace.csv" | head -1)
  python3 scripts/timeline.py $f 8 | head -4
  python3 - $O/bench_h$h.log <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"], d.get("wide_inc",{}).get("changed_rows_per_sweep"), d.get("wide_inc",{}).get("changed_arcs_per_sweep"))
PY
done
