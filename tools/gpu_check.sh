#!/bin/bash
# One GPU round: parity tests, then (if nothing crashed) a short bench.
# pytest exit 0/1 = ran (1 = some assertion failed); anything else = stop.
set -u
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-700} python -m pytest tests -m gpu -q -s ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:---steps 10 --warmup 3 --cpu-seconds 10} > gpurun_out/bench.log 2>&1
brc=$?
echo "bench rc=$brc"
tail -5 gpurun_out/bench.log
exit $brc
