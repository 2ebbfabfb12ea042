#!/bin/bash
# Two-packets-per-lane flat forms (17 / 18): parity first, then same-box A/B
# against forms 16 / 15 on Zipf frames, Zipf spans and 1500 B frames.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s3b
mkdir -p $O
cd $R
echo "start $(date)" > $O/steps.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "p2 or two_packet" > $O/pytest_p2.log 2>&1 && echo "pytest p2 ok" >> $O/steps.log && \
timeout -k 10 400 python tools/ab_kernels.py --rounds 6 --variants 16,17,15,18 --cases cfg3_zipf_frames,zipf_spans,udp1500_frames > $O/ab_forms.log 2>&1 && echo "ab forms ok" >> $O/steps.log && \
timeout -k 10 300 python tools/ab_kernels.py --rounds 6 --variants 17,17:8:0:64:1:36864,17:8:0:64:1:65536,17:8:0:64:1:98304 --cases cfg3_zipf_frames > $O/ab_p2_tiles.log 2>&1 && echo "ab tiles ok" >> $O/steps.log && \
for v in 16 17 16 17; do timeout -k 10 200 python bench.py --config mixed --steps 20 --no-cpu --variant $v >> $O/bench_mixed_ab.log 2>&1 || exit 1; done && echo "bench ab ok" >> $O/steps.log
rc=$?
echo "exit=$rc $(date)" >> $O/steps.log
tail -3 $O/pytest_p2.log
cat $O/ab_forms.log $O/ab_p2_tiles.log 2>/dev/null | grep '^{'
grep -h '^{' $O/bench_mixed_ab.log 2>/dev/null | cut -c1-300
cat $O/steps.log
exit $rc
