#!/bin/bash
# r06: the -m gpu suite at HEAD, in two calls (each under gpurun's limit):
#   scripts/gpu_suite2.sh TAG main   every -m gpu test but the full-size files, then smoke()
#   scripts/gpu_suite2.sh TAG full   the full-size files (C3 / C4 / C5 at configs' sizes, RCCL worlds)
# Output: gpurun_out/TAG/{main,full}.log (+ a heartbeat file while it runs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; mkdir -p $OUT
(while sleep 30; do date > $OUT/hb; done) &
HB=$!
trap "kill $HB" EXIT
FULL="tests/test_c3_full.py tests/test_c4_full.py tests/test_c5_full.py tests/test_rccl_world.py"
if [ "$2" = main ]; then
  DES=""; for f in $FULL; do DES="$DES --deselect $f"; done
  timeout -k 10 1000 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests $DES > $OUT/main.log 2>&1
  rc=$?; tail -3 $OUT/main.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/main.log | head; exit $rc; }
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
  rc=$?; tail -2 $OUT/smoke.log; exit $rc
else
  timeout -k 10 1050 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu $FULL > $OUT/full.log 2>&1
  rc=$?; tail -3 $OUT/full.log; [ $rc -eq 0 ] || grep -E "FAILED|Error" $OUT/full.log | head; exit $rc
fi
