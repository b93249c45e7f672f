cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python scripts/rank_probe.py 1 2 4 8 > gpurun_out/rank_probe.log 2>&1; rc=$?; cat gpurun_out/rank_probe.log | tail -12; exit $rc
