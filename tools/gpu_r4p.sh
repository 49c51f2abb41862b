#!/bin/bash
# Node-stage counter passes (round 4, after the epilogue changes; verdict r03 item 2): L2 / L1 request and hit
# counters and the SQ wait breakdown of gnn_node_kernel, one rocprofv3 --pmc
# pass per group (kernel trace only), cy-mmpde B=16 serial bench.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4p
mkdir -p $O
timeout -s KILL 60 rocprofv3 --list-avail > $O/list_avail.txt 2>&1; echo "list-avail rc=$?"
export PMC_OUT=$O PMC_REGEX="gnn_node_kernel|gnn_embed_kernel" PMC_TIMEOUT=180 \
       PMC_BENCH_ARGS="--steps 2 --warmup 1 --serial --no-f32-exact --no-cpu-baseline"
bash tools/gpu_counters.sh \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" \
  "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
  "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_REQ_sum" \
  > $O/counters.log 2>&1; rc=$?; tail -12 $O/counters.log; exit $rc
