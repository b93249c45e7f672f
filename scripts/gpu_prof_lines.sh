#!/bin/bash
# r06: rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of the default bench lines at HEAD:
# C3 (dc_multi_kernel, 512-thread workgroups) and C5 (ws_kernel). Output gpurun_out/$1/{c3,c5}/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r06pb}
(while sleep 30; do date > gpurun_out/$T.hb; done) &
HB=$!
trap "kill $HB" EXIT
mkdir -p gpurun_out
bash scripts/gpu_prof3.sh $T/c3 bench.py --no-cpu-baseline --no-refstruct --no-full-scan --no-convergence || exit $?
bash scripts/gpu_prof3.sh $T/c5 bench.py --config c5 --no-cpu-baseline --no-refstruct --no-convergence || exit $?
bash scripts/gpu_prof3.sh $T/rebuild scripts/rb_sq_probe.py || exit $?
