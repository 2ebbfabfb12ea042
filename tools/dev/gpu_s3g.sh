#!/bin/bash
# Final tree of round 2, part 2 (after gpu_s3f.sh): for every bench config a
# kernel trace plus separate FETCH_SIZE and WRITE_SIZE passes, cut to the
# timed dispatches by tools/prof_timed.py (TAG=r02 names the outputs).
# Each GPU step has its own time limit; steps chain with && (first failure ends it).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s3g
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
PROBE_BYTES=1572864000 prof udp1500 && echo "prof udp1500 ok" >> $O/steps.log && \
PROBE_BYTES=1572864000 prof fill && echo "prof fill ok" >> $O/steps.log && \
prof mixed && echo "prof mixed ok" >> $O/steps.log && \
prof tcp64k --packets 262144 && echo "prof tcp64k ok" >> $O/steps.log && \
prof slots && echo "prof slots ok" >> $O/steps.log && \
prof frags && echo "prof frags ok" >> $O/steps.log
rc=$?
echo "exit=$rc $(date)" >> $O/steps.log
cat $O/prof_*_summary.log | tail -40
cat $O/steps.log
exit $rc
