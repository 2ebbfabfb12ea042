#!/bin/bash
# Fill store-form A/B: store probe with re-read variants, fill bench with the
# whole-unit build (default) and the bytes-after-re-read build, fill parity.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02c
mkdir -p $O
cd $R
timeout -k 10 120 ./tools/dev/store_probe 3 > $O/store_probe.log 2>&1 && cat $O/store_probe.log && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fill or many_launches" > $O/pytest_fill.log 2>&1 && tail -2 $O/pytest_fill.log && \
timeout -k 10 200 python bench.py --config fill --steps 20 --no-cpu > $O/bench_fill_whole.log 2>&1 && \
SCCSUM_LIB=$R/seastar_amd/lib/libsccsum_fillbytes.so timeout -k 10 200 python bench.py --config fill --steps 20 --no-cpu > $O/bench_fill_bytes.log 2>&1 && \
timeout -k 10 200 python bench.py --config fill --steps 20 --no-cpu > $O/bench_fill_whole2.log 2>&1 && \
timeout -k 10 300 python bench.py --config sweep --no-cpu > $O/bench_sweep.log 2>&1
rc=$?
for f in $O/bench_fill_whole.log $O/bench_fill_bytes.log $O/bench_fill_whole2.log; do grep -h '^{' $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"; done
grep -h '^{' $O/bench_sweep.log | python -c "import json,sys; [print(r) for r in json.loads(sys.stdin.read())['sweep']]"
exit $rc
