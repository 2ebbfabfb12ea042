#!/bin/bash
# bench A/B: flat-kernel tile target 0 (64 packets) vs 49152 B (32 x 1500 B frames)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/ab_bench_tiles.log
: > $L
for r in 1 2; do
for c in udp1500 fill mixed; do for tb in 0 49152; do
echo -n "$c tile_bytes $tb: " >> $L
timeout -k 10 300 python bench.py --config $c --tile-bytes $tb --steps 20 --no-cpu 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'])" >> $L || exit 1
done; done; done
for tb in 0 49152; do
echo -n "tcp64k tile_bytes $tb: " >> $L
timeout -k 10 300 python bench.py --config tcp64k --tile-bytes $tb --steps 6 --no-cpu 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'])" >> $L || exit 1
done
cat $L
