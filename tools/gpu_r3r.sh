#!/bin/bash
set -u
export TMPDIR=/tmp
O=gpurun_out/r3r
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dense.py -k "chain" > $O/dense.log 2>&1
rc=$?; echo "dense rc=$rc"; grep -E "passed|failed" $O/dense.log | tail -2
grep -E "^FAILED|Error|assert" $O/dense.log | head -20
exit $rc
