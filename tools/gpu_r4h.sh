#!/bin/bash
# Round 4: BatchNorm / skinny weight-gradient kernels and training gradient tests, training-iteration kernel profile.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4h
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_rows.py tests/test_gpu_train.py tests/test_gpu_dmm_train.py -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python3 tools/train_bench.py --edge-gemm f16x3 --iters 10 --warmup 3 > $O/train_plain.json 2>&1 || { tail $O/train_plain.json; exit 6; }
tail -1 $O/train_plain.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r4h_prof -o run -- \
    python3 tools/train_bench.py --edge-gemm f16x3 --iters 5 --warmup 2 > $O/train.json 2>&1 || { tail $O/train.json; exit 5; }
f=$(find /tmp/r4h_prof -name '*kernel_stats.csv' | head -1)
cp $f $O/train_kernel_stats.csv
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total kernel ms", tot / 1e6, "per iteration (7 iterations)", tot / 7e6)
for r in rows[:45]:
    print("%-100s %5s calls avg %8.2f us  %5.2f%%" % (r["Name"][:100], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
PY
tail -1 $O/train.json
