#!/bin/bash
# Node-stage round: GNN parity subset, serial kernel stats, node-kernel counters
# (SQ issue/wait group, TCC L2 group), each GPU step under its own limit.
set -u
mkdir -p gpurun_out/r3d
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_precision.py tests/test_gpu_train.py > gpurun_out/r3d/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r3d/tests.log | tail -2
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" gpurun_out/r3d/tests.log | head; exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3d/stats -o run -- \
    python3 bench.py --steps 20 --warmup 5 --serial --no-f32-exact --no-cpu-baseline > gpurun_out/r3d/stats.log 2>&1 || exit 1
tail -1 gpurun_out/r3d/stats.log | cut -c1-300
export PMC_OUT=gpurun_out/r3d/ctr PMC_REGEX="gnn_node_kernel|gnn_embed_kernel" \
       PMC_BENCH_ARGS="--steps 2 --warmup 1 --serial --no-f32-exact --no-cpu-baseline" PMC_TIMEOUT=240
bash tools/gpu_counters.sh \
  "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
  "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_READ_sum" \
  "SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SMEM" \
  > gpurun_out/r3d/ctr.log 2>&1; echo "counters rc=$?"; tail -20 gpurun_out/r3d/ctr.log
