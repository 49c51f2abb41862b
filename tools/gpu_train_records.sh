#!/bin/bash
# Training records on the current tree: the training-iteration benches (f16x3 and exact
# fp32 edge GEMMs) and a rocprofv3 kernel summary of the f16x3 iteration.
set -u
export TMPDIR=/tmp
O=gpurun_out/${1:-train_rec}
mkdir -p $O
for m in f16x3 f32; do
  timeout -k 10 300 python3 tools/train_bench.py --edge-gemm $m --iters 10 --warmup 3 > $O/train_$m.json 2>&1 \
      || { tail $O/train_$m.json; exit 6; }
  tail -1 $O/train_$m.json
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/train_rec_prof -o run -- \
    python3 tools/train_bench.py --edge-gemm f16x3 --iters 5 --warmup 2 > $O/prof_train.json 2>&1 \
    || { tail $O/prof_train.json; exit 7; }
cp $(find /tmp/train_rec_prof -name '*kernel_stats.csv' | head -1) $O/train_kernel_stats.csv
