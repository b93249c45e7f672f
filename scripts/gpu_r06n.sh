cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/${1:-r06n}; mkdir -p $OUT
(while sleep 30; do date > $OUT/hb; done) &
HB=$!
trap "kill $HB" EXIT
MCMC_DCM_BS=512 timeout -k 5 120 python -u scripts/dcm_bs_probe.py > $OUT/probe.log 2>&1 || { tail -20 $OUT/probe.log; exit 1; }
grep "equal" $OUT/probe.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_dense.py tests/test_wide.py tests/test_knobs.py > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -3 $OUT/t.log
timeout -k 10 300 python -u scripts/wt_probe.py 10 > $OUT/wt.log 2>&1 || { tail -20 $OUT/wt.log; exit 1; }
tail -4 $OUT/wt.log | cut -c1-200
for bs in 512 1024; do
  MCMC_DCM_BS=$bs timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-refstruct --no-full-scan > $OUT/c3_bs$bs.json 2> $OUT/c3_bs$bs.err || exit 1
  echo "bs $bs: $(python3 -c "import json;d=json.loads(open('$OUT/c3_bs$bs.json').read().splitlines()[-1]);print(d['ms_per_step'], d['roofline']['kernel_ms'], d.get('convergence',{}).get('amortized_ms_per_sweep'))")"
done
timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --no-refstruct --no-convergence > $OUT/c5.json 2> $OUT/c5.err || exit 1
echo "c5: $(python3 -c "import json;d=json.loads(open('$OUT/c5.json').read().splitlines()[-1]);print(d['ms_per_step'], d['roofline']['kernel_ms'], d['wide_inc']['persistent']['step_us_per_sweep'])")"
