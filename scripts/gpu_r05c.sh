#!/bin/bash
# r05: dense tests, smoke, C3 bench line + the leader's solo trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r05c}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_dense.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/dense.log 2>&1
rc=$?; tail -3 $O/dense.log; [ $rc -ne 0 ] && { grep -n "Error\|assert\|FAIL" $O/dense.log | head -30; exit $rc; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
MCMC_SOLO_TRACE=$O/solo.bin timeout -k 10 600 python3 -u bench.py --steps 200 --warmup 0 --no-refstruct --no-cpu-baseline --no-full-scan --no-convergence > $O/c3_trace.log 2>&1 || { tail -20 $O/c3_trace.log; exit 1; }
python3 scripts/solo_trace.py $O/solo.bin
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 --no-refstruct --no-cpu-baseline --no-full-scan > $O/c3.log 2>&1 || { tail -20 $O/c3.log; exit 1; }
python3 - $O/c3.log <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print('c3', round(d['ms_per_step']*1e3,2),'us', 'kernel', d['roofline']['kernel_ms'], 'loop', d['convergence']['loop_ms'], {k: d['dense'][k] for k in ('incremental_sweeps','rebuilds','open_rows_per_sweep','moved_vertices_per_sweep')})
PY
