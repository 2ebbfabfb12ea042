#!/bin/bash
# Host wait mode A/B (bench.py --sync auto|spin), same box, alternating; then
# the run-align parity test (per-queue clamp case added).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s3h
mkdir -p $O
cd $R
echo "start $(date)" > $O/steps.log
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "run_align" > $O/pytest_align.log 2>&1 && echo "pytest ok" >> $O/steps.log && \
for m in auto spin auto spin auto spin; do timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --sync $m >> $O/bench_sync_udp1500.log 2>&1 || exit 1; done && echo "udp ok" >> $O/steps.log && \
for m in auto spin auto spin; do timeout -k 10 120 python bench.py --config mixed --steps 20 --no-cpu --sync $m >> $O/bench_sync_mixed.log 2>&1 || exit 1; done && echo "mixed ok" >> $O/steps.log && \
for m in auto spin; do timeout -k 10 120 python bench.py --steps 200 --warmup 5 --no-cpu --sync $m >> $O/bench_sync_udp1500_200.log 2>&1 || exit 1; done && echo "200 ok" >> $O/steps.log
rc=$?
echo "exit=$rc $(date)" >> $O/steps.log
tail -2 $O/pytest_align.log
for f in $O/bench_sync_*.log; do grep -h '^{' $f | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$(basename $f)', d['config']['host_wait'], d['steps'], d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"; done
cat $O/steps.log
exit $rc
