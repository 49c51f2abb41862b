#!/bin/bash
# Kernel traces of the eager three-stream step against hipGraph replay (one
# graph per stage), B = 16 and 8: tools/trace_compare.py on the timed passes
# (the bench's traced pass, 3 + 10 steps at the end, skipped).
set -u
export TMPDIR=/tmp
O=gpurun_out/${1:-graph_trace}
mkdir -p $O
for b in 16 8; do
  for g in eager graph; do
    a=""; [ $g = graph ] && a="--graph"
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t_${b}_$g -o run -- \
        python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32-exact --batch $b $a \
        > $O/b${b}_$g.json 2>&1 || { tail -20 $O/b${b}_$g.json; exit 3; }
  done
  echo "== B=$b: A = eager, B = graph"
  python3 tools/trace_compare.py $(find $O/t_${b}_eager -name '*kernel_trace.csv' | head -1) \
      $(find $O/t_${b}_graph -name '*kernel_trace.csv' | head -1) 5 1 13 | tee $O/compare_b$b.txt
done
