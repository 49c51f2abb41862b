#!/bin/bash
# Layer-kernel utilisation for DESIGN.md / profiles: three separate rocprofv3
# --pmc passes (SQ/GRBM group, FETCH_SIZE, WRITE_SIZE; kernel trace only) and
# one --kernel-trace --stats pass of the same serial bench, then
# tools/layer_counters.py joins them into gpurun_out/lc/layer_counters.json.
set -u
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --serial --no-f32-exact --no-cpu-baseline"
export PMC_OUT=gpurun_out/lc PMC_REGEX="gnn_edge_wave_kernel|gnn_node_kernel|gnn_embed_kernel|linear_skinny" \
       PMC_BENCH_ARGS="$ARGS" PMC_TIMEOUT=240
bash tools/gpu_counters.sh \
  "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES" \
  "FETCH_SIZE" "WRITE_SIZE" > gpurun_out/lc/counters.log 2>&1 || { tail -30 gpurun_out/lc/counters.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lc/stats -o run -- \
    python3 bench.py --steps 10 --warmup 3 --serial --no-f32-exact --no-cpu-baseline \
    > gpurun_out/lc/stats.log 2>&1 || { tail -20 gpurun_out/lc/stats.log; exit 1; }
python3 tools/layer_counters.py gpurun_out/lc
