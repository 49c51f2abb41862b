#!/bin/bash
# DMM GNN staging / index prefetch: DMM parity tests, full-size step, serial kernel stats.
set -u
export TMPDIR=/tmp
O=gpurun_out/r3m
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_dmm_api.py \
    tests/test_gpu_parity.py -k "dmm or mesh or full_size or moving or cells" > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "^FAILED|Error|assert" $O/tests.log | head -20; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- \
    python3 bench.py --steps 20 --warmup 5 --serial --no-f32-exact --no-cpu-baseline > $O/stats.log 2>&1 || exit 1
python3 tools/step_breakdown.py $O/stats/run_kernel_trace.csv | head -24
