#!/bin/bash
# Walk workgroup timings of the violator-heavy C5 sweep 0: light walks vs workgroup-only walks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03ah}; mkdir -p $O
timeout -k 10 300 python3 -u scripts/walk_probe.py $O/w_light.bin > $O/walk_light.log 2>&1 || exit $?
cat $O/walk_light.log
MCMC_WALK_LIGHT=0 timeout -k 10 300 python3 -u scripts/walk_probe.py $O/w_wg.bin > $O/walk_wg.log 2>&1 || exit $?
cat $O/walk_wg.log
rm -f $O/*.bin
