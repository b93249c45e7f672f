#!/bin/bash
# r06: kernel trace + FETCH_SIZE / WRITE_SIZE passes (separate runs) of one probe script, by default
# the C3 count rebuild and full-scan sweep (scripts/prof_rebuild_fullscan.py); e.g.
#   scripts/gpu_prof3.sh r06wt scripts/wt_probe.py 12
# Output: gpurun_out/$TAG/{trace,pmc1,pmc2}.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06prof}
shift
[ $# -eq 0 ] && set -- scripts/prof_rebuild_fullscan.py
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 "$@" > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -1 $OUT/trace.log | cut -c1-400
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc1 -o run -- python3 "$@" > $OUT/pmc1.log 2>&1
rc=$?; echo "pmc1 rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc2 -o run -- python3 "$@" > $OUT/pmc2.log 2>&1
rc=$?; echo "pmc2 rc=$rc"
exit $rc
