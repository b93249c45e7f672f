#!/bin/bash
# Incremental wide sweep, round 3: wide parity suite, C5 kernel timeline, SQ counters of the C5 kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03r}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_wide.py -m gpu -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
Q="--config c5 --steps 20 --warmup 5 --no-cpu-baseline --no-refstruct --no-convergence"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t1 -o run -- python3 bench.py $Q > $O/bench_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
f=$(find $O/t1 -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py $f 12
python3 scripts/trace_avg.py $f 40
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM --output-format csv -d $O/sq -o run -- python3 bench.py $Q > $O/bench_sq.log 2>&1
rc=$?; echo "sq rc=$rc"
python3 scripts/pmc_avg.py $O/sq wide_ 2>&1; python3 scripts/pmc_avg.py $O/sq commit 2>&1
exit 0
