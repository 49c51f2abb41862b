#!/bin/bash
# Round-3 micro-benchmarks: edge-kernel decomposition (random vs local
# neighbour order) and node-stage time against the row count (tail rounds).
set -u
mkdir -p gpurun_out/ub3
for m in random local; do
  timeout -k 10 90 tools/ubench/wave_diag 16 $m 24 > gpurun_out/ub3/wd_$m.log 2>&1 || exit 1
done
for B in 4 6 7 8 10 12 13 14 16 20 24 26; do
  timeout -k 10 60 tools/ubench/node_ubench $B 1 > gpurun_out/ub3/node_$B.log 2>&1 || exit 1
done
grep -h -E "production|no gathers|MFMA|bare|neighbours" gpurun_out/ub3/wd_*.log
grep -h -E "n=|RB2|RB4" gpurun_out/ub3/node_*.log
