#!/bin/bash
# Round 4: node / embed range records without the workgroup barrier (new) against HEAD (old)
set -u
O=gpurun_out/r4m
mkdir -p $O
for rep in 1 2 3; do
  for v in old new; do
    timeout -k 10 90 tools/ubench/node_phases_$v 16 > $O/$v.$rep.log 2>&1 || { tail $O/$v.$rep.log; exit 3; }
    echo "$v rep$rep: $(grep -E 'node kernel:|GEMM3|output hash|embed kernel' $O/$v.$rep.log | tr -s ' ' | tr '\n' ' ')"
  done
done
