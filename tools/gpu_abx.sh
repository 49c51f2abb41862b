#!/bin/bash
# A/B of builds of libmmpde_hip.so (mm-pde_amd/mmpde_amd/lib/ab/*.so, built
# beforehand on the CPU side): each is copied over the in-tree library in turn
# and timed with a short serial rocprofv3 kernel-trace run of bench.py; with
# AB_DUMP=1 each also dumps one cy B=16 GNN forward (tools/gnn_out_dump.py) and
# the dumps are compared bit for bit against the first build's.
set -u
export TMPDIR=/tmp
L=mm-pde_amd/mmpde_amd/lib
O=gpurun_out/${AB_OUT:-ab}
mkdir -p $O
cp $L/libmmpde_hip.so /tmp/libmmpde_hip.orig.so
for so in $L/${AB_DIR:-ab}/*.so; do
  v=$(basename $so .so)
  cp $so $L/libmmpde_hip.so
  if [ "${AB_DUMP:-0}" = 1 ]; then
    timeout -k 10 200 python3 tools/gnn_out_dump.py $O/$v.pt > $O/$v.dump.log 2>&1 || { tail -20 $O/$v.dump.log; exit 1; }
  fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- \
      python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32-exact --serial ${AB_BENCH_ARGS:-} \
      > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  f=$(find $O/$v -name '*kernel_stats.csv' | head -1)
  echo "== $v: $(grep -o '"value": [0-9.e+]*' $O/$v.log | head -1)"
  python3 - "$f" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:5]:
    print("%-60s %5s calls avg %8.1f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
cp /tmp/libmmpde_hip.orig.so $L/libmmpde_hip.so
if [ "${AB_DUMP:-0}" = 1 ]; then
  python3 - $O <<'PY'
import glob, sys, torch
fs = sorted(glob.glob(sys.argv[1] + "/*.pt"))
ref = torch.load(fs[0], weights_only=True)
for f in fs[1:]:
    d = torch.load(f, weights_only=True)
    print(f, {k: (bool(torch.equal(d[k], ref[k])), float((d[k] - ref[k]).abs().max())) for k in ref})
PY
fi
