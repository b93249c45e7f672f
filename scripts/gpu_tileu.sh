# kTileU A/B: the block probe (C3-density CSR graph, block sizes 16/15/14) and the C3 probe for the
# in-tree library and variants/libmcmc_u*.so. Usage: bash scripts/gpu_tileu.sh TAG "u5 u6"
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1; mkdir -p $O
for v in base $2; do
  if [ $v = base ]; then unset MCMC_HIP_LIB; else export MCMC_HIP_LIB=$PWD/variants/libmcmc_$v.so; fi
  PROBE_N=1400000 PROBE_VARIANTS=${PV:-16:,15:,14:} timeout -k 10 300 python -u scripts/block_probe.py > $O/bp_$v.log 2>&1 || exit $?
  grep '^{' $O/bp_$v.log | python -c "import sys,json; [print('$v', (d:=json.loads(l))['variant'], round(d['ms_per_sweep'],4), d['sub_log2'], d['C3_hash']) for l in sys.stdin]"
  if [ -z "${NOC3:-}" ]; then
    MCMC_PROBE_MODES=0 timeout -k 10 300 python -u scripts/scan_probe.py c3 > $O/c3_$v.log 2>&1 || exit $?
    echo "$v c3 $(grep '^{' $O/c3_$v.log | cut -c40-140)"
  fi
done
