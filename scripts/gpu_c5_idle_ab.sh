cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r06ab; mkdir -p $OUT
for rep in 1 2; do for p in 1 16; do
MCMC_WS_POLL_IDLE=$p timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --no-refstruct --no-convergence > $OUT/c5_$p_$rep.json 2>/dev/null || exit 1
echo "idle $p rep $rep: $(python3 -c "import json;d=json.loads(open('$OUT/c5_$p_$rep.json').read().splitlines()[-1]);print(d['ms_per_step'], d['wide_inc']['persistent']['step_us_per_sweep'])")"
done; done
