#!/bin/bash
# r05 final: C5 profile at HEAD (trace + FETCH/WRITE passes), then the bench lines (one GPU, world 1
# through the driver, a world-8 rank's share)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05w}; mkdir -p $O/c5
B="--no-cpu-baseline --no-refstruct --no-full-scan"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5/trace -o run -- python3 bench.py --config c5 --steps 20 --warmup 5 $B > $O/c5/trace.log 2>&1 || { tail -5 $O/c5/trace.log; exit 1; }
grep '^{"metric"' $O/c5/trace.log > $O/c5/bench_trace.json
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c5/pmc1 -o run -- python3 bench.py --config c5 --steps 20 --warmup 5 $B --no-convergence > $O/c5/pmc1.log 2>&1 || { tail -5 $O/c5/pmc1.log; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c5/pmc2 -o run -- python3 bench.py --config c5 --steps 20 --warmup 5 $B --no-convergence > $O/c5/pmc2.log 2>&1 || { tail -5 $O/c5/pmc2.log; exit 1; }
echo "c5 profile done"
bash scripts/gpu_r05r.sh ${1:-r05w}
