#!/bin/bash
# Round-3 measurement call: MFMA-gap filler prices (gapcost), the edge-kernel
# HBM traffic record, configs[1..2] bench lines with rocprof stats and the
# cy-gnn whole-step HBM record, and the training-iteration timing.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r3g
timeout -k 10 120 tools/ubench/gapcost > gpurun_out/r3g/gapcost.log 2>&1 || { cat gpurun_out/r3g/gapcost.log; exit 1; }
head -20 gpurun_out/r3g/gapcost.log
timeout -k 10 900 bash tools/gpu_pmc.sh > gpurun_out/r3g/pmc.log 2>&1 || { tail gpurun_out/r3g/pmc.log; exit 1; }
echo "pmc ok"
timeout -k 10 1000 bash tools/gpu_configs.sh > gpurun_out/r3g/configs.log 2>&1 || { tail gpurun_out/r3g/configs.log; exit 1; }
echo "configs ok"
timeout -k 10 700 bash tools/gpu_train.sh > gpurun_out/r3g/train.log 2>&1 || { tail gpurun_out/r3g/train.log; exit 1; }
tail -3 gpurun_out/r3g/train.log | cut -c1-300
