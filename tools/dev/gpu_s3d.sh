#!/bin/bash
# Run-start alignment (sccsum_set_run_align 1 / 4 / 8 units): parity, then
# same-box A/B on Zipf frames (odd offsets), 65 535 B spans (every tile starts
# mid-line), 1500 B frames and 64 KiB spans (already aligned), then bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s3d
mkdir -p $O
cd $R
echo "start $(date)" > $O/steps.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "run_align or full_tiles or mixed_mtu or random_layouts or every_length" > $O/pytest_align.log 2>&1 && echo "pytest ok" >> $O/steps.log && \
timeout -k 10 400 python tools/ab_kernels.py --rounds 6 --variants 16,16:8:0:64:1:49152:1:4:1:1:4,16:8:0:64:1:49152:1:4:1:1:8 --cases cfg3_zipf_frames,udp1500_frames,tcp64k_spans,tcp65535_spans > $O/ab_align.log 2>&1 && echo "ab ok" >> $O/steps.log && \
for a in 1 8 1 8; do timeout -k 10 120 python bench.py --config mixed --steps 20 --no-cpu --run-align $a >> $O/bench_mixed_ab.log 2>&1 || exit 1; done && echo "bench mixed ok" >> $O/steps.log && \
for a in 1 8; do timeout -k 10 300 python bench.py --config tcp64k --seg-len 65535 --steps 10 --no-cpu --run-align $a >> $O/bench_tcp65535_ab.log 2>&1 || exit 1; done && echo "bench tcp65535 ok" >> $O/steps.log
rc=$?
echo "exit=$rc $(date)" >> $O/steps.log
tail -3 $O/pytest_align.log
grep -h '^{' $O/ab_align.log
grep -h '^{' $O/bench_mixed_ab.log $O/bench_tcp65535_ab.log 2>/dev/null | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['metric'][-40:], d['value'], d['ms_per_step'], d['roofline']['frac'])"
cat $O/steps.log
exit $rc
