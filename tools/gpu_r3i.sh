#!/bin/bash
# Weight-stationary node kernel: ubench (timing + bitwise vs RB2), GNN parity tests, bench.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r3i
for B in 16 8; do
  timeout -k 10 90 tools/ubench/node_ubench $B 1 > gpurun_out/r3i/node_$B.log 2>&1 || { cat gpurun_out/r3i/node_$B.log; exit 1; }
  cat gpurun_out/r3i/node_$B.log
done
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_precision.py > gpurun_out/r3i/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r3i/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-exact > gpurun_out/r3i/bench.log 2>&1 || exit 1
tail -1 gpurun_out/r3i/bench.log | cut -c1-200
