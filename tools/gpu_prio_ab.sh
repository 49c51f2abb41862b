#!/bin/bash
# Stream priorities A/B (MMPDERollout.set_priorities): eager bench lines at B = 16 / 8,
# off / on / off / on, then one kernel trace per setting at B = 16 (tools/trace_compare.py).
set -u
export TMPDIR=/tmp
O=gpurun_out/${1:-prio_ab}
mkdir -p $O
for b in 16 8; do
  for p in off on off on; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-f32-exact --batch $b --priorities $p \
        > $O/b${b}_$p.json 2> $O/b${b}_$p.err || { tail $O/b${b}_$p.err; exit 3; }
    python3 -c "import json; d=json.loads(open('$O/b${b}_$p.json').read().strip().splitlines()[-1]); print('B=$b prio=$p', round(d['value']/1e6,3),'M', round(d['ms_per_step'],4),'ms host', round(d['host_issue_ms_per_step'],3))"
  done
done
for p in off on; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t_16_$p -o run -- \
      python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32-exact --priorities $p \
      > $O/t16_$p.json 2>&1 || { tail -20 $O/t16_$p.json; exit 3; }
done
python3 tools/trace_compare.py $(find $O/t_16_off -name '*kernel_trace.csv' | head -1) \
    $(find $O/t_16_on -name '*kernel_trace.csv' | head -1) 5 1 13 | tee $O/compare_b16.txt
