#!/bin/bash
# r05: persistent wide tests + C5 bench (step times)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r05i}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_wide.py tests/test_knobs.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/wide.log 2>&1
rc=$?; tail -3 $O/wide.log
if [ $rc -ne 0 ]; then grep -n "assert\|Error\|FAIL" $O/wide.log | head -30; exit $rc; fi
bash scripts/gpu_r05h.sh ${1:-r05i}
