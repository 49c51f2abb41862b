#!/bin/bash
# Round 4: node-stage A/B (phase stamps, legacy vs current build, twice), the
# kNN policy timing, GPU parity tests of the node stage, serial kernel profile.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4c
mkdir -p $O
for rep in 1 2; do
  for v in node_phases_legacy node_phases; do
    timeout -k 10 120 tools/ubench/$v 16 > $O/$v.$rep.log 2>&1 || { echo "$v failed"; cat $O/$v.$rep.log; exit 3; }
    echo "== $v rep $rep"; cat $O/$v.$rep.log
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_eval.py tests/test_gpu_api.py tests/test_time_window.py tests/test_radius.py \
    -q --timeout 240 --timeout-method thread -x > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $O/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/knn_cand_time.py 16 0.004 0.01 0.02 > $O/knn_cand_time.log 2>&1; echo "knn rc=$?"; cat $O/knn_cand_time.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32-exact --serial > $O/prof_bench.json 2>&1 \
    || { tail $O/prof_bench.json; exit 5; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
cp $f $O/kernel_stats_serial.csv
python3 - "$f" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:8]:
    print("%-60s %5s calls avg %8.2f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
tail -1 $O/prof_bench.json | cut -c1-300
