#!/bin/bash
# Quick A/B record: default bench line + serial rocprofv3 kernel summary.
# usage: tools/gpu_quick.sh TAG [extra bench args]
set -u
export TMPDIR=/tmp
T=${1:-quick}; shift || true
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 3; }
tail -1 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/q_prof -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32-exact --serial "$@" > $O/prof_bench.json 2>&1 \
    || { tail $O/prof_bench.json; exit 5; }
f=$(find /tmp/q_prof -name '*kernel_stats.csv' | head -1)
cp $f $O/kernel_stats_serial.csv
python3 - "$f" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:12]:
    print("%-60s %5s calls avg %8.2f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
