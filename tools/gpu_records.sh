#!/bin/bash
# The counter and profile records the bench line and DESIGN.md cite, one
# function per record (run on the GPU box: bash tools/gpu_records.sh <what> ...):
#   pmc NAME      the edge kernel's HBM traffic (tools/gpu_pmc.sh -> profiles/NAME.json,
#                 bench.py EDGE_PMC_RECORD) and the configs[1] / configs[2] bench lines
#                 with the cy-gnn whole-step HBM record (tools/gpu_configs.sh)
#   node          node / embed kernel counter passes (SQ wait breakdown, L2 / L1 requests)
#   train         training tests, the training-iteration bench and its kernel profile
#   bwd           edge backward kernel counter passes (SQ wait breakdown, LDS, VALU / MFMA issue)
set -u
export TMPDIR=/tmp

pmc() {
  PMC_NAME=$1 bash tools/gpu_pmc.sh || return $?
  STEP_HBM=${2:-} bash tools/gpu_configs.sh || return $?
  rm -rf gpurun_out/cfg/*.prof/*/*kernel_trace* 2>/dev/null
}

node() {
  local O=gpurun_out/node_ctr
  mkdir -p $O
  export PMC_OUT=$O PMC_REGEX="gnn_node_kernel|gnn_embed_kernel" PMC_TIMEOUT=180 \
         PMC_BENCH_ARGS="--steps 2 --warmup 1 --serial --no-f32-exact --no-cpu-baseline"
  bash tools/gpu_counters.sh \
    "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" \
    "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
    "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_REQ_sum" \
    > $O/counters.log 2>&1; local rc=$?; tail -12 $O/counters.log; return $rc
}

bwd() {
  local O=gpurun_out/bwd_ctr
  mkdir -p $O
  export PMC_OUT=$O PMC_REGEX="edge_bwd_f16_kernel" PMC_TIMEOUT=240 PMC_SCRIPT=tools/train_bench.py \
         PMC_BENCH_ARGS="--edge-gemm f16x3 --iters 1 --warmup 1"
  bash tools/gpu_counters.sh \
    "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" \
    "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES" \
    > $O/counters.log 2>&1; local rc=$?; tail -14 $O/counters.log; return $rc
}

train() {
  local O=gpurun_out/train
  mkdir -p $O
  timeout -k 10 300 python -u -m pytest tests/test_gpu_train_rows.py tests/test_gpu_train.py -q \
      --timeout 200 --timeout-method thread > $O/tests.log 2>&1
  local rc=$?; echo "pytest rc=$rc"; tail -5 $O/tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then return $rc; fi
  for m in f16x3 f32; do
    timeout -k 10 200 python3 tools/train_bench.py --edge-gemm $m --iters 10 --warmup 3 > $O/train_$m.json 2>&1 \
        || { tail $O/train_$m.json; return 6; }
    tail -1 $O/train_$m.json
  done
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/train_prof -o run -- \
      python3 tools/train_bench.py --edge-gemm f16x3 --iters 5 --warmup 2 > $O/train_prof.json 2>&1 \
      || { tail $O/train_prof.json; return 5; }
  local f=$(find /tmp/train_prof -name '*kernel_stats.csv' | head -1)
  cp $f $O/train_kernel_stats.csv
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total kernel ms", tot / 1e6, "per iteration (7 iterations)", tot / 7e6)
for r in rows[:45]:
    print("%-100s %5s calls avg %8.2f us  %5.2f%%" % (r["Name"][:100], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
PY
}

for what in "$@"; do
  case $what in
    pmc:*) pmc "${what#pmc:}" "${STEP_HBM:-}" || exit $? ;;
    node) node || exit $? ;;
    train) train || exit $? ;;
    bwd) bwd || exit $? ;;
    *) echo "unknown record $what"; exit 2 ;;
  esac
done
