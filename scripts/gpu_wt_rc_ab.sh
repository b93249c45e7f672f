# Wide tiled full sweeps: the block-major recount (default) against the mask scan (MCMC_WT_RC=0):
# parity of the tiled cases and the default-nCol C3 run, then the whole reference loop each way.
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r06wtrc; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_wide.py -k "tiled" > $OUT/t.log 2>&1; rc=$?; tail -1 $OUT/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_c3_full.py -k "default_ncol" > $OUT/t2.log 2>&1; rc=$?; tail -1 $OUT/t2.log; [ $rc -eq 0 ] || exit $rc
for cfg in "1 1000000" "1 32"; do set -- $cfg; MCMC_WT_RC=$1 MCMC_WT_ARCS_DIV=$2 timeout -k 10 300 python -u scripts/wt_loop.py > $OUT/loop_rc$1_d$2.log 2>&1 || exit 1; echo "rc $1 div $2: $(tail -1 $OUT/loop_rc$1_d$2.log | cut -c1-200)"; done
