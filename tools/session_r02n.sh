#!/bin/bash
# A/B bench --streams 1 (current stream) vs 2, same box, alternating
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/ab_bench_streams.log
: > $L
for rep in 1 2; do
for c in udp1500 mixed fill; do
for ns in 1 2; do
  echo "== $c streams $ns" >> $L
  timeout -k 10 200 python bench.py --config $c --streams $ns --steps 20 --no-cpu 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'])" >> $L || exit 1
done
done
done
cat $L
