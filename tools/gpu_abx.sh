#!/bin/bash
# A/B of builds of libmmpde_hip.so (mm-pde_amd/mmpde_amd/lib/ab/*.so, built
# beforehand on the CPU side): each is copied over the in-tree library in turn
# and timed with a short serial rocprofv3 kernel-trace run of bench.py.
set -u
export TMPDIR=/tmp
L=mm-pde_amd/mmpde_amd/lib
mkdir -p gpurun_out/${AB_OUT:-ab}
cp $L/libmmpde_hip.so /tmp/libmmpde_hip.orig.so
for so in $L/${AB_DIR:-ab}/*.so; do
  v=$(basename $so .so)
  cp $so $L/libmmpde_hip.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${AB_OUT:-ab}/$v -o run -- \
      python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32-exact --serial \
      > gpurun_out/${AB_OUT:-ab}/$v.log 2>&1 || { tail -20 gpurun_out/${AB_OUT:-ab}/$v.log; exit 1; }
  f=$(find gpurun_out/${AB_OUT:-ab}/$v -name '*kernel_stats.csv' | head -1)
  echo "== $v: $(grep -o '"value": [0-9.e+]*' gpurun_out/${AB_OUT:-ab}/$v.log | head -1)"
  python3 - "$f" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:3]:
    print("%-60s %5s calls avg %8.1f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
cp /tmp/libmmpde_hip.orig.so $L/libmmpde_hip.so
