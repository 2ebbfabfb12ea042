#!/bin/bash
# A/B: a run's first row loaded with the default cache policy (sccsum_set_head_cached 1)
# vs nontemporal (0, the default): the line shared with the previous tile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s3i
mkdir -p $O
cd $R
echo "start $(date)" > $O/steps.log
timeout -k 10 400 python tools/ab_kernels.py --rounds 8 --variants 16,16:8:0:64:1:49152:1:4:1:1:8:1 --cases cfg3_zipf_frames,udp1500_frames,tcp65535_spans > $O/ab_head.log 2>&1 && echo "ab ok" >> $O/steps.log && \
timeout -k 10 300 python tools/ab_kernels.py --rounds 8 --variants 16:8:0:64:1:49152:1:4:1:1:8:1,16 --cases cfg3_zipf_frames > $O/ab_head2.log 2>&1 && echo "ab2 ok" >> $O/steps.log
rc=$?
echo "exit=$rc $(date)" >> $O/steps.log
grep -h '^{' $O/ab_head.log $O/ab_head2.log
cat $O/steps.log
exit $rc
