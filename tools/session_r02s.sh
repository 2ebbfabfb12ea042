#!/bin/bash
# run-to-run vs box-to-box: mixed x3, udp1500 x2 (separate processes, one box)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/ab_repeat.log
: > $L
for r in 1 2 3; do for c in mixed udp1500; do
echo -n "$c run $r: " >> $L
timeout -k 10 300 python bench.py --config $c --steps 20 --no-cpu 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline'].get('measured_read_ceiling_GBps'))" >> $L || exit 1
done; done
cat $L
