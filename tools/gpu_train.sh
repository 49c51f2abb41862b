#!/bin/bash
# Training-path timing + a rocprofv3 kernel-trace --stats profile of it.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/train
mkdir -p "$OUT"
timeout -k 10 300 python3 -u tools/train_bench.py --batch ${BATCH:-16} > "$OUT/train_bench.log" 2>&1 \
    || { tail -30 "$OUT/train_bench.log"; exit 1; }
tail -1 "$OUT/train_bench.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 tools/train_bench.py --batch ${BATCH:-16} --iters 3 --warmup 1 > "$OUT/prof.log" 2>&1 \
    || { tail -30 "$OUT/prof.log"; exit 1; }
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)
head -25 "$f" | cut -c1-200
