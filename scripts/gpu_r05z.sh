#!/bin/bash
# r05 final C5 profile with the bench's default steps / warm-up (50 / 20)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05z}; mkdir -p $O/c5
B="--no-cpu-baseline --no-refstruct --no-full-scan"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5/trace -o run -- python3 bench.py --config c5 $B > $O/c5/trace.log 2>&1 || { tail -5 $O/c5/trace.log; exit 1; }
grep '^{"metric"' $O/c5/trace.log > $O/c5/bench_trace.json
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c5/pmc1 -o run -- python3 bench.py --config c5 $B --no-convergence > $O/c5/pmc1.log 2>&1 || { tail -5 $O/c5/pmc1.log; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c5/pmc2 -o run -- python3 bench.py --config c5 $B --no-convergence > $O/c5/pmc2.log 2>&1 || { tail -5 $O/c5/pmc2.log; exit 1; }
echo done
