#!/bin/bash
# r06: the bench lines at HEAD -- the default (C3, every leg), C2 and C5 -- after the dense tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r06fb}; mkdir -p $OUT
(while sleep 30; do date > $OUT/hb; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_dense.py > $OUT/t.log 2>&1
rc=$?; tail -1 $OUT/t.log; [ $rc -eq 0 ] || exit $rc
for cfg in c3 c2 c5; do
  timeout -k 10 400 python -u bench.py --config $cfg > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err || { tail -5 $OUT/bench_$cfg.err; exit 1; }
  echo "$cfg: $(python3 -c "import json;d=json.loads(open('$OUT/bench_$cfg.json').read().splitlines()[-1]);c=d.get('convergence') or {};print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], c.get('loop_ms'), c.get('rebuild_ms'), (d.get('cpu_baseline') or {}).get('value'))")"
done
