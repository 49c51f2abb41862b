#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -s -k "knn or full_size" --timeout 300 --timeout-method thread > gpurun_out/knn_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/knn_tests.log | tail -2; grep -E "^FAILED|^ERROR" gpurun_out/knn_tests.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python tools/knn_cand_time.py 16 0.004 0.02 0.08 > gpurun_out/knn_cand_time.log 2>&1 || exit 1
timeout -k 10 200 python tools/host_overhead.py 16 20 > gpurun_out/host_overhead.log 2>&1 || exit 1
head -3 gpurun_out/host_overhead.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-exact > gpurun_out/bench.log 2>&1 || exit 1
tail -1 gpurun_out/bench.log | cut -c1-250
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-exact --graph > gpurun_out/bench_graph.log 2>&1 || exit 1
tail -1 gpurun_out/bench_graph.log | cut -c1-250
