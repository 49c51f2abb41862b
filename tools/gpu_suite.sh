#!/bin/bash
# -m gpu suite (optionally a -k filter) then the quick bench + serial profile.
# usage: tools/gpu_suite.sh TAG [pytest -k expr]
set -u
export TMPDIR=/tmp
T=${1:-suite}; K=${2:-}
O=gpurun_out/$T
mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -v -rP --timeout 240 --timeout-method thread -k "$K" > $O/gpu_tests.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1
fi
rc=$?
echo "pytest rc=$rc"; tail -15 $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_quick.sh $T/q
