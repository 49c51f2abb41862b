#!/bin/bash
# GPU tests, kNN candidate timings, bench, serial rocprof stats.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -3; grep -E "^FAILED|^ERROR" gpurun_out/gpu_tests.log | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python tools/knn_cand_time.py 16 0.004 0.02 0.08 > gpurun_out/knn_cand_time.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit 1
tail -1 gpurun_out/bench.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_serial -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --serial > gpurun_out/bench_serial.log 2>&1
echo "prof rc=$?"
