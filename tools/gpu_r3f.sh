#!/bin/bash
# Full GPU test suite + bench + serial kernel stats (round-3 small-kernel changes).
set -u
mkdir -p gpurun_out/r3f
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests -m gpu \
    > gpurun_out/r3f/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r3f/tests.log | tail -2
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" gpurun_out/r3f/tests.log | head -20; exit $rc; fi
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3f/bench.log 2>&1 || exit 1
tail -1 gpurun_out/r3f/bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3f/stats -o run -- \
    python3 bench.py --steps 20 --warmup 5 --serial --no-f32-exact --no-cpu-baseline > gpurun_out/r3f/stats.log 2>&1 || exit 1
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/r3f/stats/run_kernel_stats.csv')))
for r in rows[:24]:
    print(f"{float(r['TotalDurationNs'])/1e3/50:8.1f} us/step {int(r['Calls'])/50:5.2f}/step avg {float(r['AverageNs'])/1e3:7.1f}  {r['Name'][:70]}")
PY
