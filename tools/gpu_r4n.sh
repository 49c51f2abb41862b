#!/bin/bash
# Round 4: edge kernel with the W2 image staged once per 4-wave workgroup (new)
# against HEAD (old): wave_diag timing + fp64 check (ab_run.sh), node_phases
# output hashes (the edge sums feed the node stage), and the bench line with
# either library, alternating.
set -u
O=gpurun_out/r4n
mkdir -p $O
for rep in 1 2; do for v in old new; do LD_LIBRARY_PATH=tools/ubench/libab/$v timeout -k 10 120 tools/ubench/wave_diag 16 > $O/wd_$v.$rep.log 2>&1 || exit 1; echo "wave_diag $v $rep: $(grep -E "^production" $O/wd_$v.$rep.log)"; done; done
for v in old new; do
  timeout -k 10 90 tools/ubench/node_phases_$v 16 > $O/np_$v.log 2>&1 || { tail $O/np_$v.log; exit 2; }
  echo "$v: $(grep -E 'output hash|embed kernel' $O/np_$v.log | tr -s ' ' | tr '\n' ' ')"
done
LIB=mm-pde_amd/mmpde_amd/lib/libmmpde_hip.so
for rep in 1 2; do
  for v in old new; do
    cp tools/ubench/libab/$v/libmmpde_hip.so $LIB || exit 4
    timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-f32-exact \
        > $O/bench_$v.$rep.json 2> $O/bench_$v.$rep.err || { tail $O/bench_$v.$rep.err; exit 3; }
    python3 -c "
import json; d=json.loads(open('$O/bench_$v.$rep.json').read().strip().splitlines()[-1])
print('$v', $rep, round(d['value']/1e6,3), round(d['ms_per_step'],4), 'edge', round(d['roofline']['launch_ms']*1e3,2), 'node', round(d['node_stage_ms']*1e3,2))"
  done
done
cp tools/ubench/libab/new/libmmpde_hip.so $LIB
