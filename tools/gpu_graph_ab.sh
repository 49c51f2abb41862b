#!/bin/bash
# Eager three-stream step against hipGraph replay of the same step (bench.py --graph) at
# 16, 8 and 4 trajectories: the eager step's host issue time is ~0.9 ms, so the smaller
# batches (configs[4]'s 8-GPU end point runs 8 per rank) may be host-bound.
set -u
O=gpurun_out/graph_ab; mkdir -p $O
for b in 16 8 4; do
  for g in "" "--graph"; do
    n=b$b${g:+_graph}
    timeout -k 10 300 python -u bench.py --steps 30 --batch $b $g --no-cpu-baseline --no-f32-exact > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 3; }
    python3 -c "
import json,sys; r=json.loads(open('$O/$n.json').read().strip().splitlines()[-1])
print('$n', 'value %.3fM ms %.3f host %.3f edge %.1f node %.1f' % (r['value']/1e6, r['ms_per_step'], r['host_issue_ms_per_step'], r['roofline']['launch_ms']*1e3, r['node_stage_ms']*1e3))"
  done
done
