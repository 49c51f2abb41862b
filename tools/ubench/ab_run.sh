#!/bin/bash
# A/B of library builds under tools/ubench/ab/<name>/libmmpde_hip.so with the
# wave_diag edge-kernel bench (production line + fp64 check), interleaved twice.
set -u
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for d in tools/ubench/ab/*/; do
    v=$(basename $d)
    LD_LIBRARY_PATH=$d timeout -k 10 120 tools/ubench/wave_diag 16 > gpurun_out/ab/$v.$rep.log 2>&1 || { tail -5 gpurun_out/ab/$v.$rep.log; exit 1; }
    echo "$v rep$rep: $(grep -E '^production|vs fp64' gpurun_out/ab/$v.$rep.log | tr -s ' ' | tr '\n' ' ')"
  done
done
