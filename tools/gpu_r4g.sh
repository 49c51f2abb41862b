#!/bin/bash
# Round 4: conv weight-gradient tests, training-iteration kernel profile.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_cnn.py tests/test_gpu_dmm_train.py -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r4g_prof -o run -- \
    python3 tools/train_bench.py --edge-gemm f16x3 --iters 5 --warmup 2 > $O/train.json 2>&1 || { tail $O/train.json; exit 5; }
f=$(find /tmp/r4g_prof -name '*kernel_stats.csv' | head -1)
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
