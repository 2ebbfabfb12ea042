#!/bin/bash
# Row kernel with the next step's metadata prefetched: parity on the row
# kernel, then bench --config slots alternating the previous library
# (seastar_amd/lib/ab/libsccsum_base.so) and this tree's.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s3e
mkdir -p $O
cd $R
echo "start $(date)" > $O/steps.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "rows" > $O/pytest_rows.log 2>&1 && echo "pytest ok" >> $O/steps.log && \
for i in 1 2 3; do \
  SCCSUM_LIB=$R/seastar_amd/lib/ab/libsccsum_base.so timeout -k 10 120 python bench.py --config slots --steps 20 --no-cpu >> $O/bench_slots_base.log 2>&1 && \
  timeout -k 10 120 python bench.py --config slots --steps 20 --no-cpu >> $O/bench_slots_new.log 2>&1 || exit 1; done && echo "bench ok" >> $O/steps.log
rc=$?
echo "exit=$rc $(date)" >> $O/steps.log
tail -3 $O/pytest_rows.log
for f in base new; do grep -h '^{' $O/bench_slots_$f.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'])"; done
cat $O/steps.log
exit $rc
