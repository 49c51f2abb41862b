#!/bin/bash
# kNN-30 query fp32-first sort: kNN parity tests, full-size step parity, serial kernel stats.
set -u
export TMPDIR=/tmp
O=gpurun_out/r3k
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "knn or full_size or burgers" > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|Error|assert" $O/tests.log | head -20; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- \
    python3 bench.py --steps 20 --warmup 5 --serial --no-f32-exact --no-cpu-baseline > $O/stats.log 2>&1 || exit 1
python3 tools/step_breakdown.py $O/stats/run_kernel_trace.csv | head -20
timeout -k 10 200 python3 tools/knn_cand_time.py 16 0.004 0.02 > $O/knn_cand_time.log 2>&1 || exit 1
cat $O/knn_cand_time.log | tail -12
