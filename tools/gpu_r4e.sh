#!/bin/bash
# Round 4: training-iteration kernel profile (f16x3) and the node-side GEMM shapes.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 300 python -u tools/gemm_shapes.py > $O/gemm_shapes.log 2>&1; echo "gemm rc=$?"; cat $O/gemm_shapes.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 tools/train_bench.py --edge-gemm f16x3 --iters 5 --warmup 2 > $O/train.json 2>&1 || { tail $O/train.json; exit 5; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
cp $f $O/train_kernel_stats.csv
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total kernel ms", tot / 1e6)
for r in rows[:40]:
    print("%-100s %5s calls avg %8.2f us  %5.2f%%" % (r["Name"][:100], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
PY
