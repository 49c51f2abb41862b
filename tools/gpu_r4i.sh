#!/bin/bash
# Round 4: edge-backward placement A/B (tools/ubench/bwd_ab.cpp variants).
set -u
O=gpurun_out/r4i
mkdir -p $O
for rep in 1; do
  for v in base; do
    echo "== $v rep $rep" >> $O/bwd_ab.log
    timeout -k 10 120 tools/ubench/bwd_ab_$v >> $O/bwd_ab.log 2>&1 || { tail -5 $O/bwd_ab.log; exit 3; }
  done
done
cat $O/bwd_ab.log
