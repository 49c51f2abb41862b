#!/bin/bash
# 16-row range records + node RB3 / residual-in-registers variants: ubench, parity tests.
set -u
export TMPDIR=/tmp
O=gpurun_out/r3l
mkdir -p $O
for B in 16 8; do
  timeout -k 10 120 tools/ubench/node_ubench $B 1 > $O/node_$B.log 2>&1 || { cat $O/node_$B.log; exit 1; }
  cat $O/node_$B.log
done
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_precision.py tests/test_gpu_eval.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|Error|assert" $O/tests.log | head -20; exit $rc; }
