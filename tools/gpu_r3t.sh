#!/bin/bash
# fp16x3 edge backward: edge / training-step gradient tests, then the training
# bench in both modes.
set -u
export TMPDIR=/tmp
O=gpurun_out/r3t
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_train.py > $O/train_tests.log 2>&1
rc=$?; echo "train tests rc=$rc"; grep -E "passed|failed" $O/train_tests.log | tail -2
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error|assert" $O/train_tests.log | head -20; exit $rc; fi
for m in f32 f16x3; do
  timeout -k 10 300 python3 -u tools/train_bench.py --edge-gemm $m > $O/train_bench_$m.log 2>&1 || { tail -20 $O/train_bench_$m.log; exit 1; }
  tail -1 $O/train_bench_$m.log
done
