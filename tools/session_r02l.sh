#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02l
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && tail -1 $O/pytest_gpu.log && \
timeout -k 10 300 python bench.py --config fill --steps 20 --no-cpu > $O/bench_fill.log 2>&1 && \
timeout -k 10 300 python bench.py --config sweep --no-cpu > $O/bench_sweep.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log
grep -h '^{' $O/bench_fill.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('fill', d['value'], r['avg_launch_us'], r['frac'])"
grep -h '^{' $O/bench_sweep.log | python -c "import json,sys; [print(r) for r in json.loads(sys.stdin.read())['sweep']]"
exit $rc
