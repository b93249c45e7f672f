#!/bin/bash
# r05: world-1 driver batches as persistent launches: multi-GPU tests, then the world-1 bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r05s}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_multi.py tests/test_knobs.py tests/test_distributed.py -k "not test_wide_knobs and not test_tiled_scan_knobs" > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
tail -2 $O/t.log
for cfg in c3 c2 c5; do
  timeout -k 10 400 python -u bench.py --config $cfg --force-dist --steps 40 --warmup 5 --no-cpu-baseline --no-refstruct --no-convergence > $O/bench_${cfg}_dist1.log 2>&1 || { tail -5 $O/bench_${cfg}_dist1.log; exit 1; }
  grep '^{"metric"' $O/bench_${cfg}_dist1.log > $O/bench_${cfg}_dist1.json
  python3 -c "
import json; d=json.loads(open('$O/bench_${cfg}_dist1.json').read()); print('$cfg dist1', round(d['ms_per_step']*1e3,2), 'us/step, device', round(d['roofline']['kernel_ms']*1e3,2))"
done
