#!/bin/bash
# Walk workgroup timings of the violator-heavy C5 sweep 0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r03ab}; mkdir -p $O
timeout -k 10 300 python3 -u scripts/walk_probe.py $O/walk.phase > $O/walk.log 2>&1
rc=$?; cat $O/walk.log | grep -v amdgpu.ids; exit $rc
