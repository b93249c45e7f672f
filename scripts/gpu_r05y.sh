#!/bin/bash
# r05 final C5: wide + multi tests, the C5 profile (trace, FETCH/WRITE), the C5 bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05y}; mkdir -p $O/c5
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_wide.py tests/test_multi.py tests/test_knobs.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
B="--no-cpu-baseline --no-refstruct --no-full-scan"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5/trace -o run -- python3 bench.py --config c5 --steps 20 --warmup 5 $B > $O/c5/trace.log 2>&1 || { tail -5 $O/c5/trace.log; exit 1; }
grep '^{"metric"' $O/c5/trace.log > $O/c5/bench_trace.json
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c5/pmc1 -o run -- python3 bench.py --config c5 --steps 20 --warmup 5 $B --no-convergence > $O/c5/pmc1.log 2>&1 || { tail -5 $O/c5/pmc1.log; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c5/pmc2 -o run -- python3 bench.py --config c5 --steps 20 --warmup 5 $B --no-convergence > $O/c5/pmc2.log 2>&1 || { tail -5 $O/c5/pmc2.log; exit 1; }
timeout -k 10 400 python -u bench.py --config c5 > $O/bench_c5.log 2>&1 || { tail -5 $O/bench_c5.log; exit 1; }
grep '^{"metric"' $O/bench_c5.log > $O/bench_c5.json
timeout -k 10 400 python -u bench.py --config c5 --force-dist --steps 40 --warmup 5 --no-cpu-baseline --no-refstruct --no-convergence > $O/bench_c5_dist1.log 2>&1 || { tail -5 $O/bench_c5_dist1.log; exit 1; }
grep '^{"metric"' $O/bench_c5_dist1.log > $O/bench_c5_dist1.json
python3 -c "
import json
for f in ('bench_c5','bench_c5_dist1'):
    d=json.loads(open('$O/'+f+'.json').read()); h=d.get('headline') or {}
    print(f, round(d['ms_per_step']*1e3,2), 'us', round(d['roofline']['kernel_ms']*1e3,2), (h.get('violator_sweeps') or {}).get('ms_per_sweep'))"
