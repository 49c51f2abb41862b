#!/bin/bash
# Final round-3 pass: node early-U2 A/B, full GPU suite + bench + serial
# profile (r3x), training bench in both modes.
set -u
export TMPDIR=/tmp
bash tools/gpu_ab_node.sh || exit 1
R3Q_OUT=r3x bash tools/gpu_r3q.sh || exit 1
O=gpurun_out/r3x
for m in f32 f16x3; do
  timeout -k 10 300 python3 -u tools/train_bench.py --edge-gemm $m > $O/train_bench_$m.log 2>&1 || { tail -20 $O/train_bench_$m.log; exit 1; }
  tail -1 $O/train_bench_$m.log
done
