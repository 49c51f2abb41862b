set -u
# Round 4: DPP max reductions in segment_range (edge kernels' prologue): node_phases hashes (the
# edge sums feed the node stage) of HEAD~ (old) and HEAD (new), then one bench line.
O=gpurun_out/r4q; mkdir -p $O
for v in old new; do timeout -k 10 90 tools/ubench/node_phases_$v 16 > $O/np_$v.log 2>&1 || exit 2; echo "$v: $(grep -E 'output hash|embed kernel' $O/np_$v.log | tr -s ' ' | tr '\n' ' ')"; done
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-f32-exact > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 3; }
python3 -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print(round(d['value']/1e6,3), round(d['ms_per_step'],4), 'edge', round(d['roofline']['launch_ms']*1e3,2), 'node', round(d['node_stage_ms']*1e3,2))"
