#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02i
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && tail -2 $O/pytest_gpu.log && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_multi.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --launch single > $O/bench_single.log 2>&1 && \
timeout -k 10 300 python bench.py --config sweep --no-cpu > $O/bench_sweep.log 2>&1
rc=$?
tail -20 $O/pytest_gpu.log | grep -E "passed|failed|Error|error" | head
for f in $O/bench_multi.log $O/bench_single.log; do grep -h '^{' $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'], r['measured_read_ceiling_GBps'])"; done
grep -h '^{' $O/bench_sweep.log | python -c "import json,sys; [print(r) for r in json.loads(sys.stdin.read())['sweep']]"
exit $rc
