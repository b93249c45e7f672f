#!/bin/bash
# Tie-binade word-function walk: wide parity + full-size C5, per-task walk timings, violator loop, C5 line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03aj}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_wide.py tests/test_c5_full.py -m gpu -x -q -p no:cacheprovider \
    --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u scripts/walk_probe.py $O/w.bin > $O/walk.log 2>&1 || exit $?
grep -v amdgpu.ids $O/walk.log; rm -f $O/w.bin
for i in 1 2; do
  timeout -k 10 300 python3 scripts/c5_viol_probe.py > $O/viol_$i.log 2>&1 || exit $?
  echo "$(grep rep $O/viol_$i.log | tr '\n' ' ' | cut -c1-220)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tv -o run -- python3 scripts/c5_viol_probe.py > $O/viol_t.log 2>&1 || exit $?
python3 scripts/viol_trace.py $(find $O/tv -name "*kernel_trace.csv" | head -1) 12
timeout -k 10 600 python -u bench.py --config c5 > $O/bench_c5.log 2>&1 || exit $?
grep '^{' $O/bench_c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', d['ms_per_step'], d['value'], d.get('violators'))"
