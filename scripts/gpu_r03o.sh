#!/bin/bash
# Incremental wide sweep: the wide + partitioned parity suites, then the C5 bench line (short legs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r03o}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_wide.py tests/test_rmat.py -m gpu -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
Q="--no-refstruct --no-cpu-baseline"
for m in 1 0; do
  MCMC_WIDE_INC=$m timeout -k 10 600 python -u bench.py --config c5 $Q > $O/bench_c5_inc$m.log 2>&1
  rc=$?; echo "bench c5 inc=$m rc=$rc"; tail -1 $O/bench_c5_inc$m.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
  python - $O/bench_c5_inc$m.log <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print({k: d.get(k) for k in ("ms_per_step",)}, d.get("violators"), d.get("headline",{}).get("reference_loop"), d.get("wide_inc"))
PY
done
