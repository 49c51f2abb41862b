#!/bin/bash
# gpu_quick.sh, then a rocprofv3 kernel-trace --stats pass of a short serial
# bench (per-kernel averages): gpurun_out/quick/prof.
set -u
export TMPDIR=/tmp
bash tools/gpu_quick.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/quick/prof -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32-exact --serial \
    > gpurun_out/quick/prof.log 2>&1 || { tail -20 gpurun_out/quick/prof.log; exit 1; }
f=$(find gpurun_out/quick/prof -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:14]:
    print("%-70s %5s calls avg %8.1f us  %5.1f%%" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
PY
