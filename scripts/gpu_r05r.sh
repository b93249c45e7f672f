#!/bin/bash
# r05: bench lines at HEAD -- one GPU (c3 / c2 / c5, full default legs), world 1 through the driver
# (--force-dist), and one world-8 rank's share of C3 (--rank-share 8)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r05r}; mkdir -p $O
for cfg in c3 c2 c5; do
  timeout -k 10 400 python -u bench.py --config $cfg > $O/bench_$cfg.log 2>&1 || { tail -5 $O/bench_$cfg.log; exit 1; }
  grep '^{"metric"' $O/bench_$cfg.log > $O/bench_$cfg.json; echo "$cfg $(cut -c1-160 $O/bench_$cfg.json)"
  timeout -k 10 400 python -u bench.py --config $cfg --force-dist --steps 40 --warmup 5 --no-cpu-baseline --no-refstruct --no-convergence > $O/bench_${cfg}_dist1.log 2>&1 || { tail -5 $O/bench_${cfg}_dist1.log; exit 1; }
  grep '^{"metric"' $O/bench_${cfg}_dist1.log > $O/bench_${cfg}_dist1.json; echo "$cfg dist1 $(cut -c1-160 $O/bench_${cfg}_dist1.json)"
done
timeout -k 10 400 python -u bench.py --rank-share 8 --steps 40 --warmup 5 > $O/share8.log 2>&1 || { tail -5 $O/share8.log; exit 1; }
grep '^{' $O/share8.log | tail -1 > $O/share8.json; cut -c1-300 $O/share8.json
