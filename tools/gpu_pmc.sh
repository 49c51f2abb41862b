#!/bin/bash
# HBM traffic of the dominant kernel: two separate rocprofv3 --pmc passes
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; no --sys-trace /
# runtime-trace beside --pmc), then tools/pmc_summary.py turns the per-dispatch
# counters into profiles/<name>.json (per-launch bytes, gfx950 FETCH_SIZE x2
# correction from MI355X_MICROARCH.md §HBM).
set -u
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc}
REGEX=${PMC_REGEX:-gnn_layer_fused}
ARGS=${PMC_BENCH_ARGS:---steps 2 --warmup 1 --no-cpu-baseline --no-f32-exact}
mkdir -p "$OUT"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 ${PMC_TIMEOUT:-300} rocprofv3 --pmc $c --kernel-include-regex "$REGEX" \
      --output-format csv -d "$OUT/$c" -o run -- python3 bench.py $ARGS > "$OUT/$c.log" 2>&1
  rc=$?
  echo "pmc $c rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$c.log"; exit $rc; fi
done
python3 tools/pmc_summary.py "$OUT" ${PMC_NAME:-edge_pmc}
