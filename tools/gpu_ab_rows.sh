#!/bin/bash
# A/B (A B A B) of library builds in mm-pde_amd/mmpde_amd/lib/abx/*.so on the
# row-GEMM timings (tools/rgemm_bench.py) and the training iteration
# (tools/train_bench.py, f16x3; its loss must match across builds).
set -u
L=mm-pde_amd/mmpde_amd/lib
O=gpurun_out/abr
mkdir -p $O
cp $L/libmmpde_hip.so /tmp/libmmpde_hip.orig.so
for rep in 1 2; do
for so in $L/abx/*.so; do
  v=$(basename $so .so)_$rep
  cp $so $L/libmmpde_hip.so
  echo "== $v"
  timeout -k 10 120 python3 -u tools/rgemm_bench.py > $O/$v.rg.log 2>&1 || { tail $O/$v.rg.log; cp /tmp/libmmpde_hip.orig.so $L/libmmpde_hip.so; exit 1; }
  python3 -c "
import json,sys
for l in open('$O/$v.rg.log'):
    if l.startswith('{'):
        d=json.loads(l); print('  ', d['k'], d['nout'], 'fwd', d['fwd_us'], 'dx', d['dx_us'], 'dw', d['dw_us'])
"
  timeout -k 10 200 python3 tools/train_bench.py --edge-gemm f16x3 --iters 20 > $O/$v.train.json 2>&1 || { tail $O/$v.train.json; cp /tmp/libmmpde_hip.orig.so $L/libmmpde_hip.so; exit 2; }
  tail -1 $O/$v.train.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('   train', d['ms_per_iter'], 'loss', repr(d['loss']))"
done
done
cp /tmp/libmmpde_hip.orig.so $L/libmmpde_hip.so
