#!/bin/bash
# Kernel split of the training iteration with the fp16x3 edge backward.
set -u
export TMPDIR=/tmp
O=gpurun_out/r3w
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- \
    python3 tools/train_bench.py --edge-gemm f16x3 --iters 3 --warmup 1 > $O/train.log 2>&1 || { tail -20 $O/train.log; exit 1; }
tail -1 $O/train.log
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r3w/stats/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:90]}')
PY
