#!/bin/bash
# Final tree of round 2 (run starts on 128 B lines), part 1: GPU suite, smoke,
# every bench config.  Part 2 (gpu_s3g.sh) takes the profiler passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s3f
mkdir -p $O
cd $R
echo "start $(date)" > $O/steps.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo "pytest ok" >> $O/steps.log && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo "smoke ok" >> $O/steps.log && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 12 > $O/bench_udp1500.log 2>&1 && echo "bench ok" >> $O/steps.log && \
timeout -k 10 300 python bench.py --config fill --steps 20 --no-cpu > $O/bench_fill.log 2>&1 && echo "fill ok" >> $O/steps.log && \
timeout -k 10 300 python bench.py --config mixed --steps 20 --no-cpu > $O/bench_mixed.log 2>&1 && echo "mixed ok" >> $O/steps.log && \
timeout -k 10 400 python bench.py --config tcp64k --steps 10 --no-cpu > $O/bench_tcp64k.log 2>&1 && echo "tcp64k ok" >> $O/steps.log && \
timeout -k 10 400 python bench.py --config tcp64k --seg-len 65535 --steps 10 --no-cpu > $O/bench_tcp65535.log 2>&1 && echo "tcp65535 ok" >> $O/steps.log && \
timeout -k 10 300 python bench.py --config sweep --no-cpu > $O/bench_sweep.log 2>&1 && echo "sweep ok" >> $O/steps.log && \
timeout -k 10 300 python bench.py --config e2e --steps 5 --no-cpu > $O/bench_e2e.log 2>&1 && echo "e2e ok" >> $O/steps.log && \
timeout -k 10 300 python bench.py --config mixed --align 64 --steps 20 --no-cpu > $O/bench_mixed_align64.log 2>&1 && echo "mixed align64 ok" >> $O/steps.log && \
timeout -k 10 300 python bench.py --config slots --steps 20 --no-cpu > $O/bench_slots.log 2>&1 && echo "slots ok" >> $O/steps.log && \
timeout -k 10 300 python bench.py --config frags --steps 20 --no-cpu > $O/bench_frags.log 2>&1 && echo "frags ok" >> $O/steps.log
rc=$?
echo "exit=$rc $(date)" >> $O/steps.log
tail -2 $O/pytest_gpu.log
for f in $O/bench_*.log; do grep -h '^{' $f | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); r=d.get('roofline') or {}; print('$(basename $f)', d['value'], d['ms_per_step'], r.get('frac'), r.get('avg_launch_us'))" 2>/dev/null; done
cat $O/steps.log
exit $rc
