#!/bin/bash
# Bench lines of BASELINE configs[1] (burgers-mmpde) and configs[2] (cy-gnn),
# each with its CPU baseline, a rocprofv3 kernel-trace --stats run, and for
# cy-gnn (the "scatter-add / HBM roofline" config) the whole-step HBM bytes
# from two --pmc passes.  Output under gpurun_out/cfg.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/cfg
mkdir -p "$OUT"
for cfg in cy-gnn burgers-mmpde; do
  timeout -k 10 300 python3 -u bench.py --config $cfg --cpu-seconds ${CPU_SECONDS:-12} > "$OUT/$cfg.bench.log" 2>&1 \
      || { tail -20 "$OUT/$cfg.bench.log"; exit 1; }
  grep '^{' "$OUT/$cfg.bench.log" | tail -1 > "$OUT/$cfg.bench.json"
  echo "$cfg bench ok"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$cfg.prof" -o run -- \
      python3 bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-f32-exact --serial \
      > "$OUT/$cfg.prof.log" 2>&1 || { tail -20 "$OUT/$cfg.prof.log"; exit 1; }
  echo "$cfg prof ok"
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc/$c" -o run -- python3 bench.py \
      --config cy-gnn --steps 2 --warmup 1 --no-cpu-baseline --no-f32-exact --serial > "$OUT/pmc.$c.log" 2>&1 \
      || { tail -20 "$OUT/pmc.$c.log"; exit 1; }
done
python3 tools/step_hbm.py "$OUT/${STEP_HBM:-r03_cy_gnn_step_hbm}.json" cy-gnn 20168 6 "$OUT/pmc"
