#!/bin/bash
# C2 phase split (MCMC_PHASE_DUMP) and pair trace on the current build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r03ae}; mkdir -p $O
MCMC_PROBE_MODES=0 MCMC_PHASE_DUMP=$O/c2.phase timeout -k 10 300 python -u scripts/scan_probe.py c2 > $O/c2probe.log 2>&1 || exit $?
grep '^{' $O/c2probe.log | cut -c1-120
python3 scripts/phase_summary.py $O/c2.phase
timeout -k 10 300 python -u scripts/pair_probe.py c2 $O/c2 > $O/c2pair.log 2>&1 || exit $?
cat $O/c2pair.log | grep -v amdgpu; python3 scripts/pair_trace_summary.py $O/c2.trace
