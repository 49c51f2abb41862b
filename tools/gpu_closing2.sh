#!/bin/bash
# Closing GPU pass, part 2 (part 1 = the -m gpu suite + smoke, run as its own call):
# the default bench line, the configs[4] strong-scaling line at one GPU (64
# trajectories), a serial rocprofv3 kernel trace of the default bench, the
# training-iteration benches (f16x3 and exact fp32 edge GEMMs) and the configs[0-2]
# lines.  Stops at the first crash / timeout.
set -u
export TMPDIR=/tmp
O=gpurun_out/${1:-closing}
mkdir -p $O
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
for m in f16x3 f32; do
  timeout -k 10 300 python3 tools/train_bench.py --edge-gemm $m --iters 10 --warmup 3 > $O/train_$m.json 2>&1 \
      || { tail $O/train_$m.json; exit 6; }
  tail -1 $O/train_$m.json
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/closing_train_prof -o run -- \
    python3 tools/train_bench.py --edge-gemm f16x3 --iters 5 --warmup 2 > $O/prof_train.json 2>&1 \
    || { tail $O/prof_train.json; exit 7; }
f=$(find /tmp/closing_train_prof -name '*kernel_stats.csv' | head -1)
cp $f $O/train_kernel_stats.csv
for cfg in cy-gnn burgers-mmpde burgers-gnn; do
  timeout -k 10 300 python3 -u bench.py --config $cfg > $O/$cfg.bench.log 2>&1 || { tail -20 $O/$cfg.bench.log; exit 8; }
  grep '^{' $O/$cfg.bench.log | tail -1 > $O/$cfg.bench.json
  echo "$cfg bench ok"
done
