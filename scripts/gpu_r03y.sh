#!/bin/bash
# Violator-heavy C5 loop: kernel timelines with and without the incremental counts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03y}; mkdir -p $O
for m in 1 0; do
  MCMC_WIDE_INC=$m timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tv$m -o run -- python3 scripts/c5_viol_probe.py > $O/viol$m.log 2>&1
  rc=$?; echo "viol inc=$m rc=$rc"; grep rep $O/viol$m.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
