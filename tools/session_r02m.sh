#!/bin/bash
# desc kernel with per-lane metadata loads: tests, burst modes, timeline
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_desc.py tests/test_gpu_burst.py tests/test_cpp_api.py -m gpu > gpurun_out/m_tests.log 2>&1 || { tail -40 gpurun_out/m_tests.log; exit 1; }
tail -2 gpurun_out/m_tests.log
L=gpurun_out/burst_modes.log
: > $L
for rep in 1 2; do
for args in "4 1000000 mapped 32 2" "4 1000000 mapped 32 1" "4 1000000 mapped 32 0" "2 1000000 mapped 32 2" "8 1000000 mapped 32 2"; do
  $T 60 ./build/burst_gpu 8000000 $args >> $L 2>&1 || { echo "FAIL $args rc=$?" >> $L; cat $L; exit 1; }
done
done
grep -v OK $L
$T 200 python -u tools/desc_probe.py 16384 10 > gpurun_out/desc_probe.log 2>&1 || { cat gpurun_out/desc_probe.log; exit 1; }
cat gpurun_out/desc_probe.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in 2 0; do
$T 120 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/bt$m -o run --output-format csv -- ./build/burst_gpu 2000000 4 1000000 mapped 32 $m > gpurun_out/bt$m.log 2>&1 || exit 1
done
python3 tools/burst_timeline.py gpurun_out/bt2 gpurun_out/bt0 > gpurun_out/burst_timeline.txt
cat gpurun_out/burst_timeline.txt
