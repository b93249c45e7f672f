#!/bin/bash
# r06: SQ counters of the count rebuild (scripts/rb_sq_probe.py), one pass per counter set.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06sq}; mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 scripts/rb_sq_probe.py > $OUT/trace.log 2>&1 || exit $?
echo trace ok
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS --output-format csv -d $OUT/sq1 -o run -- python3 scripts/rb_sq_probe.py > $OUT/sq1.log 2>&1 || exit $?
echo sq1 ok
timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/sq2 -o run -- python3 scripts/rb_sq_probe.py > $OUT/sq2.log 2>&1 || exit $?
echo sq2 ok
