#!/bin/bash
# Closing GPU pass (regenerates the r04_final* records): the -m gpu suite, smoke(), the default bench line,
# the configs[4] strong-scaling line at one GPU (64 trajectories), a serial
# rocprofv3 kernel trace of the default bench, the training-iteration benches
# (f16x3 and exact fp32 edge GEMMs) and the configs[1] / configs[2] lines.
# Stops at the first crash / timeout.
set -u
export TMPDIR=/tmp
O=gpurun_out/closing
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -v --timeout 240 --timeout-method thread \
    > $O/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -6 $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 2; }
echo "smoke ok"
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 3; }
tail -1 $O/bench.json
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --global-trajectories 64 --no-cpu-baseline \
    > $O/bench_g64.json 2> $O/bench_g64.err || { tail $O/bench_g64.err; exit 4; }
tail -1 $O/bench_g64.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/closing_prof -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32-exact --serial > $O/prof_bench.json 2>&1 \
    || { tail $O/prof_bench.json; exit 5; }
f=$(find /tmp/closing_prof -name '*kernel_stats.csv' | head -1)
cp $f $O/kernel_stats_serial.csv
python3 - "$f" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:8]:
    print("%-60s %5s calls avg %8.2f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
for m in f16x3 f32; do
  timeout -k 10 300 python3 tools/train_bench.py --edge-gemm $m --iters 10 --warmup 3 > $O/train_$m.json 2>&1 \
      || { tail $O/train_$m.json; exit 6; }
  tail -1 $O/train_$m.json
done
for cfg in cy-gnn burgers-mmpde burgers-gnn; do
  timeout -k 10 300 python3 -u bench.py --config $cfg > $O/$cfg.bench.log 2>&1 || { tail -20 $O/$cfg.bench.log; exit 7; }
  grep '^{' $O/$cfg.bench.log | tail -1 > $O/$cfg.bench.json
  echo "$cfg bench ok"
done
