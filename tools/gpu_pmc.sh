#!/bin/bash
# HBM traffic of the dominant kernel (the GNN edge stage): separate rocprofv3
# --pmc passes for FETCH_SIZE and WRITE_SIZE (they cannot share a pass on
# gfx950; no --sys-trace / runtime-trace beside --pmc), for both arithmetic
# modes, then tools/pmc_summary.py writes gpurun_out/pmc/<name>.json (per-launch
# bytes, gfx950 FETCH_SIZE x2 correction from MI355X_MICROARCH.md §HBM) in the
# format bench.py reads as roofline.traffic.
set -u
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc}
REGEX=${PMC_REGEX:-gnn_edge_kernel|gnn_edge_wave_kernel}
mkdir -p "$OUT"
for mode in f16x3 f32; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 ${PMC_TIMEOUT:-300} rocprofv3 --pmc $c --kernel-include-regex "$REGEX" \
        --output-format csv -d "$OUT/$mode/$c" -o run -- python3 bench.py --steps 2 --warmup 1 \
        --no-cpu-baseline --no-f32-exact --edge-gemm $mode > "$OUT/$mode.$c.log" 2>&1
    rc=$?
    echo "pmc $mode $c rc=$rc"
    if [ $rc -ne 0 ]; then tail -20 "$OUT/$mode.$c.log"; exit $rc; fi
  done
done
python3 tools/pmc_summary.py ${PMC_NAME:-edge_pmc_r03} cy-mmpde 40336 f16x3="$OUT/f16x3" f32="$OUT/f32"
