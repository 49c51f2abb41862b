#!/bin/bash
# Round-3 check: edge locality experiment, GPU tests, kNN candidate timings, bench.
set -u
mkdir -p gpurun_out
for m in random local self; do
  timeout -k 10 60 tools/ubench/wave_diag 16 $m 24 > gpurun_out/wd_$m.log 2>&1 || exit 1
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python tools/knn_cand_time.py 16 0.004 0.02 0.08 > gpurun_out/knn_cand_time.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1
echo "bench rc=$?"; tail -3 gpurun_out/bench.log
