#!/bin/bash
# Round 4: update_net_1's mean-half operands issued with the h-half ones in the
# last layer's node kernel (MMPDE_NODE_EARLY_M=1, em1) against the default (base)
set -u
O=gpurun_out/r4t
mkdir -p $O
for rep in 1 2 3; do
  for v in base em1; do
    timeout -k 10 90 tools/ubench/node_phases_$v 16 > $O/$v.$rep.log 2>&1 || { tail $O/$v.$rep.log; exit 3; }
    echo "$v rep$rep: $(grep -E 'node kernel:|output hash' $O/$v.$rep.log | sed 's/the stamped launch spans [0-9.]* us//' | tr -s ' ' | tr '\n' ' ')"
  done
done
