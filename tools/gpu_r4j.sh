#!/bin/bash
# Round 4: this round's records for bench.py -- the edge kernel's HBM traffic
# (tools/gpu_pmc.sh -> edge_pmc_r04) -- and the configs[1] / configs[2] bench
# lines with the cy-gnn whole-step HBM record (tools/gpu_configs.sh ->
# r04_cy_gnn_step_hbm).
set -u
export TMPDIR=/tmp
PMC_NAME=edge_pmc_r04 bash tools/gpu_pmc.sh || exit $?
STEP_HBM=r04_cy_gnn_step_hbm bash tools/gpu_configs.sh || exit $?
rm -rf gpurun_out/cfg/*.prof/*/*kernel_trace* 2>/dev/null
du -sh gpurun_out
