#!/bin/bash
# Whole GPU suite (now with the two-packet forms 17 / 18), smoke, default
# bench, then the same-box A/B of forms 17 / 18 against 16 / 15.  Forms 17 / 18
# lost (profiles/r02_ab_p2.log) and were removed: this script records the run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s3c
mkdir -p $O
cd $R
echo "start $(date)" > $O/steps.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo "pytest ok" >> $O/steps.log && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo "smoke ok" >> $O/steps.log && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 6 > $O/bench.log 2>&1 && echo "bench ok" >> $O/steps.log && \
timeout -k 10 300 python tools/ab_kernels.py --rounds 6 --variants 16,17,15,18 --cases cfg3_zipf_frames,zipf_spans,udp1500_frames > $O/ab_forms.log 2>&1 && echo "ab forms ok" >> $O/steps.log && \
timeout -k 10 200 python tools/ab_kernels.py --rounds 6 --variants 17,17:8:0:64:1:36864,17:8:0:64:1:65536 --cases cfg3_zipf_frames > $O/ab_p2_tiles.log 2>&1 && echo "ab tiles ok" >> $O/steps.log && \
for v in 16 17 16 17; do timeout -k 10 120 python bench.py --config mixed --steps 20 --no-cpu --variant $v >> $O/bench_mixed_ab.log 2>&1 || exit 1; done && echo "bench ab ok" >> $O/steps.log
rc=$?
echo "exit=$rc $(date)" >> $O/steps.log
tail -3 $O/pytest_gpu.log
cat $O/ab_forms.log $O/ab_p2_tiles.log 2>/dev/null | grep '^{'
grep -h '^{' $O/bench.log $O/bench_mixed_ab.log 2>/dev/null | cut -c1-300
cat $O/steps.log
exit $rc
