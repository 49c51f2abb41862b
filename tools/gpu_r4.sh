#!/bin/bash
# Round-4 GPU pass: the -m gpu suite, the default bench line, the configs[4]
# strong-scaling line at one GPU (64 trajectories), and a serial rocprofv3
# kernel trace of the default bench.  Stops at the first crash / timeout.
set -u
export TMPDIR=/tmp
O=gpurun_out/${R4_TAG:-r4}
mkdir -p $O
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -q -v --timeout 240 --timeout-method thread \
      ${PYTEST_ARGS:-} > $O/gpu_tests.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -15 $O/gpu_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 3; }
tail -1 $O/bench.json
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --global-trajectories 64 --no-cpu-baseline \
    > $O/bench_g64.json 2> $O/bench_g64.err || { tail $O/bench_g64.err; exit 4; }
tail -1 $O/bench_g64.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32-exact --serial > $O/prof_bench.json 2>&1 \
    || { tail $O/prof_bench.json; exit 5; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
cp $f $O/kernel_stats_serial.csv
python3 - "$f" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:12]:
    print("%-60s %5s calls avg %8.2f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
