#!/bin/bash
# fill store pass A/B: field stores vs 64-B line rewrites
set -o pipefail
mkdir -p gpurun_out/r02q
O=gpurun_out/r02q
for r in 1 2; do for f in 0 1; do
echo -n "fill-store $f: "
timeout -k 10 300 python bench.py --config fill --fill-store $f --steps 20 --no-cpu 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'])" || exit 1
done; done
