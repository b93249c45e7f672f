#!/bin/bash
# r05 profiles at HEAD: FETCH/WRITE calibration probe, then per config a rocprofv3 kernel trace +
# stats of a short bench and the FETCH_SIZE / WRITE_SIZE passes (separate runs, no other domains)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05n}; mkdir -p $O/calib
timeout -k 10 120 ./scripts/fetch_probe > $O/calib/probe.log 2>&1 || { cat $O/calib/probe.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/calib/pmc1 -o run -- ./scripts/fetch_probe > $O/calib/p1.log 2>&1 || { tail -5 $O/calib/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/calib/pmc2 -o run -- ./scripts/fetch_probe > $O/calib/p2.log 2>&1 || { tail -5 $O/calib/p2.log; exit 1; }
python3 scripts/fetch_calib.py $O/calib $O/calib/fetch_calib.json || exit 1
for cfg in ${CFGS:-c3 c2 c5}; do
  extra=""; [ $cfg = c2 ] && extra="--config c2"; [ $cfg = c5 ] && extra="--config c5"; [ $cfg = c3 ] && extra="--config c3"
  B="--no-cpu-baseline --no-refstruct --no-full-scan"; mkdir -p $O/$cfg
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$cfg/trace -o run -- python3 bench.py $extra --steps 20 --warmup 5 $B > $O/$cfg/trace.log 2>&1 || { tail -5 $O/$cfg/trace.log; exit 1; }
  tail -1 $O/$cfg/trace.log > $O/$cfg/bench_trace.json
  timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$cfg/pmc1 -o run -- python3 bench.py $extra --steps 20 --warmup 5 $B --no-convergence > $O/$cfg/pmc1.log 2>&1 || { tail -5 $O/$cfg/pmc1.log; exit 1; }
  timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/$cfg/pmc2 -o run -- python3 bench.py $extra --steps 20 --warmup 5 $B --no-convergence > $O/$cfg/pmc2.log 2>&1 || { tail -5 $O/$cfg/pmc2.log; exit 1; }
  echo "$cfg done: $(cut -c1-200 $O/$cfg/bench_trace.json)"
done
