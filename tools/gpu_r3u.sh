#!/bin/bash
# Chain A/B (standalone and in the bench step), then the node-stage counters.
set -u
export TMPDIR=/tmp
O=gpurun_out/r3u
mkdir -p $O
timeout -k 10 200 python3 -u tools/chain_ab.py > $O/chain_ab.log 2>&1 || { tail -20 $O/chain_ab.log; exit 1; }
tail -1 $O/chain_ab.log
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-f32-exact --chain > $O/bench_chain.log 2>&1 || { tail -20 $O/bench_chain.log; exit 1; }
grep '^{' $O/bench_chain.log | tail -1 | cut -c1-200
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-f32-exact > $O/bench_nochain.log 2>&1 || { tail -20 $O/bench_nochain.log; exit 1; }
grep '^{' $O/bench_nochain.log | tail -1 | cut -c1-200
