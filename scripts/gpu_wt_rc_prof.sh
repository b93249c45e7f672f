# Kernel-time breakdown of the default-nCol C3 reference loop with the recount full sweeps.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/r06wtrc_prof; mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 -u scripts/wt_loop.py > $OUT/loop.log 2>&1 || exit 1
f=$(ls $OUT/prof/run_kernel_stats.csv 2>/dev/null | head -n 1); [ -n "$f" ] && cut -d, -f1-7 "$f" | cut -c1-60,100-220 | sed -n "1,16p"; true
