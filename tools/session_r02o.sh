#!/bin/bash
# full GPU tests + smoke, and the SURVEY §8(d) layout variants: cfg 3 (ii) 64 B-aligned, cfg 4 65535 B
set -o pipefail
mkdir -p gpurun_out/r02o
O=gpurun_out/r02o
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py --config mixed --align 64 --steps 20 --no-cpu > $O/bench_mixed_align64.log 2>&1 || { tail $O/bench_mixed_align64.log; exit 1; }
timeout -k 10 400 python bench.py --config tcp64k --seg-len 65535 --steps 10 --no-cpu > $O/bench_tcp65535.log 2>&1 || { tail $O/bench_tcp65535.log; exit 1; }
grep -h '^{' $O/bench_*.log | cut -c1-700
