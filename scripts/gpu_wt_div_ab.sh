cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r06wtd; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_wide.py -k "tiled" > $OUT/t.log 2>&1; rc=$?; tail -1 $OUT/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_c3_full.py -k "default_ncol" > $OUT/t2.log 2>&1; rc=$?; tail -1 $OUT/t2.log; [ $rc -eq 0 ] || exit $rc
for d in 2 4; do MCMC_WT_ARCS_DIV=$d timeout -k 10 300 python -u scripts/wt_loop.py > $OUT/loop_$d.log 2>&1 || exit 1; echo "div $d: $(tail -1 $OUT/loop_$d.log | cut -c1-200)"; done
