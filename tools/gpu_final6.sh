#!/bin/bash
# Round-6 final6 pass: the weight-gradient row GEMM A/B (tools/ubench/tn_ab_*:
# the committed rgemm.hip against the working tree, output hashes must match),
# then the -m gpu suite, smoke, the default bench line and the training benches
# with a kernel-trace profile of the f16x3 iteration.  Stops at the first failure.
set -u
export TMPDIR=/tmp
O=gpurun_out/${1:-final6}
mkdir -p $O
for v in head base head base; do
  echo "== $v"; timeout -k 10 60 tools/ubench/tn_ab_$v || exit 2
done > $O/tn_ab.log 2>&1
cat $O/tn_ab.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 3; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 4; }
tail -2 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 5; }
tail -1 $O/bench.json
for m in f16x3 f32; do
  timeout -k 10 300 python3 tools/train_bench.py --edge-gemm $m --iters 20 --warmup 3 > $O/train_$m.json 2>&1 \
      || { tail $O/train_$m.json; exit 6; }
  tail -1 $O/train_$m.json
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/final6_train_prof -o run -- \
    python3 tools/train_bench.py --edge-gemm f16x3 --iters 5 --warmup 2 > $O/prof_train.json 2>&1 \
    || { tail $O/prof_train.json; exit 7; }
f=$(find /tmp/final6_train_prof -name '*kernel_stats.csv' | head -1)
cp $f $O/train_kernel_stats.csv
echo done
