#!/bin/bash
# Quick C5 iteration: wide tests, the c5 bench (no CPU legs), a commit phase dump and a kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-c5q}
timeout -k 10 400 python -u -m pytest tests/test_wide.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c5q_tests.log 2>&1
rc=$?; echo "wide tests rc=$rc"; tail -3 gpurun_out/c5q_tests.log; [ $rc -ne 0 ] && exit $rc
if [ -n "$SUITE" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
MCMC_PHASE_DUMP=gpurun_out/c5_phase.bin timeout -k 10 300 python -u bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --no-refstruct > gpurun_out/bench_c5q.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_c5q.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
python scripts/phase_summary.py gpurun_out/c5_phase.bin | head -3
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --config c5 --steps 20 --warmup 2 --no-cpu-baseline --no-refstruct > $OUT/bench_trace.log 2>&1
rc=$?; echo "trace rc=$rc"
python3 - $OUT/trace/run_kernel_trace.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
out = [(r['Kernel_Name'].split('(')[0].replace('mcmc::', '').replace('void ', ''),
        (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000) for r in rows
       if 'wide' in r['Kernel_Name'] or 'commit' in r['Kernel_Name']]
for i in range(len(out) - 10, len(out), 5):
    print('  '.join(f"{a[:12]} {b:7.1f}" for a, b in out[i:i + 5]))
PY
exit $rc
