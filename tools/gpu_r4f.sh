#!/bin/bash
# Round 4: training-path tests (GNN + BaseCNN) and the training-iteration bench.
set -u
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_cnn.py -v -s --timeout 300 --timeout-method thread \
    > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed" $O/tests.log | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for m in f16x3 f32; do
  timeout -k 10 300 python -u tools/train_bench.py --edge-gemm $m > $O/train_$m.json 2>&1; echo "train $m rc=$?"; tail -1 $O/train_$m.json
done
