#!/bin/bash
# Round-2 GPU session (final tree: nt result stores, verify-only rx halves): parity tests, every bench config, and for udp1500 /
# mixed / fill / tcp64k a kernel trace plus separate FETCH_SIZE and WRITE_SIZE
# passes, cut to the timed dispatches by tools/prof_timed.py.
# Each GPU step has its own time limit; steps chain with && (first failure ends it).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r02b}
mkdir -p $O
cd $R
export TMPDIR=/tmp
STEPS_PROF="--steps 10 --warmup 2 --no-cpu"
prof() {  # prof <config> <extra bench args...>: trace + FETCH + WRITE passes, then the cut
    local c=$1; shift
    cd /tmp && \
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$c/trace -o run --output-format csv -- python3 $R/bench.py --config $c $STEPS_PROF "$@" > $O/prof_${c}_trace.log 2>&1 && \
    timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/prof_$c/fetch -o run --output-format csv -- python3 $R/bench.py --config $c $STEPS_PROF "$@" > $O/prof_${c}_fetch.log 2>&1 && \
    timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/prof_$c/write -o run --output-format csv -- python3 $R/bench.py --config $c $STEPS_PROF "$@" > $O/prof_${c}_write.log 2>&1 && \
    cd $R && python tools/prof_timed.py --bench-log $O/prof_${c}_trace.log --trace $O/prof_$c/trace \
        --fetch $O/prof_$c/fetch --write $O/prof_$c/write --probe-bytes ${PROBE_BYTES:-0} --config $c \
        --label "${TAG:-r02b} bench.py --config $c $STEPS_PROF $*" \
        --out $O/${TAG:-r02b}_pmc_$c.json --trace-out $O/${TAG:-r02b}_trace_$c.csv > $O/prof_${c}_summary.log 2>&1
}
echo "start $(date)" > $O/steps.log
[ -n "$SKIP_PYTEST" ] || timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo "pytest ok" >> $O/steps.log && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 12 > $O/bench.log 2>&1 && echo "bench ok" >> $O/steps.log && \
timeout -k 10 300 python bench.py --config fill --steps 20 --no-cpu > $O/bench_fill.log 2>&1 && echo "fill ok" >> $O/steps.log && \
timeout -k 10 300 python bench.py --config mixed --steps 20 --no-cpu > $O/bench_mixed.log 2>&1 && echo "mixed ok" >> $O/steps.log && \
timeout -k 10 400 python bench.py --config tcp64k --steps 10 --no-cpu > $O/bench_tcp64k.log 2>&1 && echo "tcp64k ok" >> $O/steps.log && \
timeout -k 10 300 python bench.py --config sweep --no-cpu > $O/bench_sweep.log 2>&1 && echo "sweep ok" >> $O/steps.log && \
timeout -k 10 300 python bench.py --config e2e --steps 5 --no-cpu > $O/bench_e2e.log 2>&1 && echo "e2e ok" >> $O/steps.log && \
timeout -k 10 300 python bench.py --steps 20 --no-cpu --rx-out2 > $O/ab_rx_out2.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --no-cpu >> $O/ab_rx_out2.log 2>&1 && \
timeout -k 10 300 python bench.py --config mixed --steps 20 --no-cpu --launch multi --rx-out2 >> $O/ab_rx_out2.log 2>&1 && \
timeout -k 10 300 python bench.py --config mixed --steps 20 --no-cpu --launch multi >> $O/ab_rx_out2.log 2>&1 && \
timeout -k 10 300 python bench.py --config mixed --steps 20 --no-cpu >> $O/ab_rx_out2.log 2>&1 && echo "ab rx_out2 ok" >> $O/steps.log && \
timeout -k 10 300 python bench.py --config mixed --align 64 --steps 20 --no-cpu > $O/bench_mixed_align64.log 2>&1 && echo "mixed align64 ok" >> $O/steps.log && \
timeout -k 10 300 python bench.py --config slots --steps 20 --no-cpu > $O/bench_slots.log 2>&1 && echo "slots ok" >> $O/steps.log && \
timeout -k 10 300 python bench.py --config frags --steps 20 --no-cpu > $O/bench_frags.log 2>&1 && echo "frags ok" >> $O/steps.log && \
PROBE_BYTES=1572864000 prof udp1500 && echo "prof udp1500 ok" >> $O/steps.log && \
PROBE_BYTES=1572864000 prof fill && echo "prof fill ok" >> $O/steps.log && \
prof mixed && echo "prof mixed ok" >> $O/steps.log && \
prof tcp64k --packets 262144 && echo "prof tcp64k ok" >> $O/steps.log && \
prof slots && echo "prof slots ok" >> $O/steps.log && \
prof frags && echo "prof frags ok" >> $O/steps.log
rc=$?
echo "exit=$rc $(date)" >> $O/steps.log
grep -h '^{' $O/bench*.log | cut -c1-400
cat $O/steps.log
exit $rc
