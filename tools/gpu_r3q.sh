#!/bin/bash
# Linear chains (res_cut, DMM output MLP + P in one launch each): dense tests
# first, then the full GPU suite, the default bench line and a serial profile.
set -u
export TMPDIR=/tmp
O=gpurun_out/${R3Q_OUT:-r3q}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dense.py > $O/dense.log 2>&1
rc=$?; echo "dense rc=$rc"; grep -E "passed|failed" $O/dense.log | tail -2
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error|assert" $O/dense.log | head -20; exit $rc; fi
timeout -k 10 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" $O/tests.log | tail -2
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error|assert" $O/tests.log | head -20; exit $rc; fi
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 > $O/bench.json; cut -c1-300 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- \
    python3 bench.py --steps 20 --warmup 5 --serial --no-f32-exact --no-cpu-baseline > $O/stats.log 2>&1 || exit 1
python3 tools/step_breakdown.py $O/stats/run_kernel_trace.csv | head -24
