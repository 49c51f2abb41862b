#!/bin/bash
# A/B (A B A B) of library builds in mm-pde_amd/mmpde_amd/lib/abx/*.so: the
# node / embed kernel means of a short serial rocprofv3 run of bench.py each.
set -u
export TMPDIR=/tmp
L=mm-pde_amd/mmpde_amd/lib
O=gpurun_out/abn
mkdir -p $O
cp $L/libmmpde_hip.so /tmp/libmmpde_hip.orig.so
for rep in 1 2; do
for so in $L/abx/*.so; do
  v=$(basename $so .so)_$rep
  cp $so $L/libmmpde_hip.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- \
      python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32-exact --serial \
      > $O/$v.log 2>&1 || { tail -20 $O/$v.log; cp /tmp/libmmpde_hip.orig.so $L/libmmpde_hip.so; exit 1; }
  f=$(find $O/$v -name '*kernel_stats.csv' | head -1)
  echo "== $v: $(grep -o '"ms_per_step": [0-9.e+]*' $O/$v.log | head -1)"
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if any(s in r["Name"] for s in ("gnn_node_kernel", "gnn_embed_kernel", "gnn_edge_wave")):
        print("   %-50s %5s calls avg %8.2f us" % (r["Name"][:50], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
done
cp /tmp/libmmpde_hip.orig.so $L/libmmpde_hip.so
