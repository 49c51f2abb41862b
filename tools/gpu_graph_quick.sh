#!/bin/bash
# Eager vs graph-replay bench lines at B = 16 / 8 / 4 (no CPU baseline, no f32 pass).
set -u
export TMPDIR=/tmp
O=gpurun_out/${1:-graphq}
mkdir -p $O
for b in 16 8 4; do
  for g in "" "--graph" "--graph=serial"; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-f32-exact --batch $b $g > $O/b$b$g.json 2> $O/b$b$g.err \
      || { tail $O/b$b$g.err; exit 3; }
    python3 -c "import json,sys; d=json.loads(open('$O/b$b$g.json').read().strip().splitlines()[-1]); print('B=$b', '$g' or 'eager', round(d['value']/1e6,3),'M', round(d['ms_per_step'],4),'ms', 'edge', round(d['roofline']['launch_ms']*1e3,1),'us host', round(d['host_issue_ms_per_step'],3))"
  done
done
