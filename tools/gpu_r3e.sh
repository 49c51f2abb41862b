#!/bin/bash
# GNN parity + serial kernel stats (node-stage iteration).
set -u
mkdir -p gpurun_out/r3e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_precision.py tests/test_gpu_eval.py > gpurun_out/r3e/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r3e/tests.log | tail -2
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" gpurun_out/r3e/tests.log | head; exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3e/stats -o run -- \
    python3 bench.py --steps 20 --warmup 5 --serial --no-f32-exact --no-cpu-baseline > gpurun_out/r3e/stats.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32-exact > gpurun_out/r3e/bench.log 2>&1 || exit 1
tail -1 gpurun_out/r3e/bench.log | cut -c1-250
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/r3e/stats/run_kernel_stats.csv')))
for r in rows[:10]:
    print(f"{float(r['AverageNs'])/1e3:8.1f} us  calls {r['Calls']:>5}  {r['Name'][:80]}")
PY
