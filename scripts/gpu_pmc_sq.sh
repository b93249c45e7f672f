# SQ/LDS counters of the C3 early-exit sweep (one pass: 8 SQ + 1 GRBM), then a summary per kernel.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
CTRS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
MCMC_PROBE_MODES=${MODES:-0} timeout -s KILL 240 rocprofv3 --pmc $CTRS --output-format csv -d $O/sq -o run -- python3 scripts/scan_probe.py ${CFG:-c3} > $O/sq.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 scripts/pmc_avg.py $O/sq sweep_tiled
