#!/bin/bash
# zero-copy pipeline: tests + cfg 5 variants, C++ batch program
set -o pipefail
mkdir -p gpurun_out/r02p
O=gpurun_out/r02p
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_cpp_api.py tests/test_gpu_desc.py -m gpu -k "pipeline or cpp or desc" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --config e2e --steps 8 --no-cpu > $O/bench_e2e.log 2>&1 || { tail $O/bench_e2e.log; exit 1; }
grep -h '^{' $O/bench_e2e.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value']); [print(k,v) for k,v in d['variants'].items()]"
