#!/bin/bash
# head_cached mode 2 (first row cached only in single-packet-tile launches) vs 0,
# on 64 KiB and 65 535 B spans; both orders.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s3k
mkdir -p $O
cd $R
echo "start $(date)" > $O/steps.log
timeout -k 10 400 python tools/ab_kernels.py --rounds 10 --variants 16,16:8:0:64:1:49152:1:4:1:1:8:2 --cases tcp64k_spans,tcp65535_spans > $O/ab.log 2>&1 && echo "ab ok" >> $O/steps.log && \
timeout -k 10 400 python tools/ab_kernels.py --rounds 10 --variants 16:8:0:64:1:49152:1:4:1:1:8:2,16 --cases tcp64k_spans,tcp65535_spans > $O/ab2.log 2>&1 && echo "ab2 ok" >> $O/steps.log
rc=$?
echo "exit=$rc $(date)" >> $O/steps.log
grep -h '^{' $O/ab.log $O/ab2.log
cat $O/steps.log
exit $rc
