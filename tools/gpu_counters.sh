#!/bin/bash
# One rocprofv3 --pmc pass per counter group (kernel-trace only; never combined
# with sys/runtime traces), restricted to kernels matching $PMC_REGEX.
# Usage: tools/gpu_counters.sh "GRP1" "GRP2" ...   (each GRP = space-separated counters)
set -u
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/ctr}
REGEX=${PMC_REGEX:-gnn_layer_fused}
ARGS=${PMC_BENCH_ARGS:---steps 2 --warmup 1 --no-cpu-baseline --no-f32-exact}
SCRIPT=${PMC_SCRIPT:-bench.py}   # or tools/train_bench.py (PMC_BENCH_ARGS its arguments)
mkdir -p "$OUT"
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 ${PMC_TIMEOUT:-300} rocprofv3 --pmc $grp --kernel-include-regex "$REGEX" \
      --output-format csv -d "$OUT/g$i" -o run -- python3 $SCRIPT $ARGS > "$OUT/g$i.log" 2>&1
  rc=$?
  echo "pmc group $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/g$i.log"; exit $rc; fi
done
python3 tools/ctr_summary.py "$OUT"
