#!/bin/bash
# Round 4: rollout bench of the r04_v1 commit (worktree _ab_old) against HEAD on
# one box, alternating, twice each (box-to-box clock spread is several %).
set -u
O=gpurun_out/r4ab
mkdir -p $O
for rep in 1 2; do
  for v in old new; do
    d=.; [ $v = old ] && d=_ab_old
    (cd $d && timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-f32-exact) \
        > $O/$v.$rep.json 2> $O/$v.$rep.err || { tail $O/$v.$rep.err; exit 3; }
    python3 -c "
import json; d=json.loads(open('$O/$v.$rep.json').read().strip().splitlines()[-1])
print('$v', $rep, round(d['value']/1e6,3), round(d['ms_per_step'],4), 'edge', round(d['roofline']['launch_ms']*1e3,2), 'node', round(d['node_stage_ms']*1e3,2))"
  done
done
