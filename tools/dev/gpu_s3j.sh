#!/bin/bash
# Zipf tile size with line-aligned run starts: 64 (cap, default), 48, 32 packets per tile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s3j
mkdir -p $O
cd $R
echo "start $(date)" > $O/steps.log
timeout -k 10 400 python tools/ab_kernels.py --rounds 8 --variants 16,16:8:0:48,16:8:0:32 --cases cfg3_zipf_frames,zipf_spans > $O/ab_tiles.log 2>&1 && echo "ab ok" >> $O/steps.log && \
timeout -k 10 300 python tools/ab_kernels.py --rounds 8 --variants 16:8:0:32,16:8:0:48,16 --cases cfg3_zipf_frames > $O/ab_tiles2.log 2>&1 && echo "ab2 ok" >> $O/steps.log
rc=$?
echo "exit=$rc $(date)" >> $O/steps.log
grep -h '^{' $O/ab_tiles.log $O/ab_tiles2.log
cat $O/steps.log
exit $rc
