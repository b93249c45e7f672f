cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/pytest_gpu.log
cp /root/repo/scripts_keep_u8.so /tmp/old.so 2>/dev/null
for v in new old; do
  if [ $v = new ]; then L=mcmc_colorer_amd/libmcmc_hip.so; else L=mcmc_colorer_amd/build/libmcmc_old.so; fi
  MCMC_HIP_LIB=$L timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/b_$v.log 2>&1 || exit 1
  MCMC_HIP_LIB=$L timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmcA_$v -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || exit 2
  MCMC_HIP_LIB=$L timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcB_$v -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || exit 3
done
python - <<'PY'
import json, csv, collections
for v in ['new','old']:
    d=json.loads(open('gpurun_out/b_%s.log'%v).read().strip().splitlines()[-1]); print(v, '%.3e'%d['value'], '%.4f ms'%d['roofline']['kernel_ms'], '%.3f'%d['roofline']['frac'])
    for p in ['pmcA','pmcB']:
        rows=list(csv.DictReader(open('gpurun_out/%s_%s/run_counter_collection.csv'%(p,v))))
        agg=collections.defaultdict(list)
        for r in rows:
            if 'sweep_kernel' in r['Kernel_Name']: agg[r['Counter_Name']].append(float(r['Counter_Value']))
        print('  ', {k: '%.3e'%(sum(x)/len(x)) for k,x in agg.items()})
PY
