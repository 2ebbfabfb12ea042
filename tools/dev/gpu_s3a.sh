#!/bin/bash
# Session-3 check of the restored tree: GPU parity tests, smoke, default bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s3a
mkdir -p $O
cd $R
echo "start $(date)" > $O/steps.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo "pytest ok" >> $O/steps.log && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo "smoke ok" >> $O/steps.log && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 && echo "bench ok" >> $O/steps.log && \
timeout -k 10 300 python bench.py --config mixed --steps 20 --no-cpu > $O/bench_mixed.log 2>&1 && echo "mixed ok" >> $O/steps.log
rc=$?
echo "exit=$rc $(date)" >> $O/steps.log
tail -3 $O/pytest_gpu.log
grep -h '^{' $O/bench*.log | cut -c1-600
cat $O/steps.log
exit $rc
