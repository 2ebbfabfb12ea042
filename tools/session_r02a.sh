#!/bin/bash
# Round-2 first GPU session: GPU tests, the store-cost probe, a profiled bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02a_gputest.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r02a_gputest.log; exit 1; }
tail -3 gpurun_out/r02a_gputest.log
timeout -k 10 120 ./tools/dev/store_probe 3 > gpurun_out/r02a_store_probe.log 2>&1 || { echo "store probe failed"; cat gpurun_out/r02a_store_probe.log; exit 1; }
cat gpurun_out/r02a_store_probe.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02a_prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r02a_bench_prof.log 2>&1 || { echo "profiled bench failed"; tail -30 gpurun_out/r02a_bench_prof.log; exit 1; }
grep '^{' gpurun_out/r02a_bench_prof.log
