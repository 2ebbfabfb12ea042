#!/bin/bash
# cfg 4 at full size (2 M x 64 KiB segments per GPU, the bench's own launch):
# kernel trace + FETCH_SIZE + WRITE_SIZE passes cut to the timed dispatches,
# then the cfg 4 bench lines (64 KiB and 65 535 B) reading that profile.
# Each GPU step has its own time limit; steps chain with && (first failure ends it).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s3l
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
prof tcp64k && echo "prof tcp64k ok" >> $O/steps.log && \
cp $O/${TAG:-r02b}_pmc_tcp64k.json $R/profiles/ && \
timeout -k 10 400 python bench.py --config tcp64k --steps 10 --no-cpu > $O/bench_tcp64k.log 2>&1 && echo "tcp64k ok" >> $O/steps.log && \
timeout -k 10 400 python bench.py --config tcp64k --seg-len 65535 --steps 10 --no-cpu > $O/bench_tcp65535.log 2>&1 && echo "tcp65535 ok" >> $O/steps.log
rc=$?
echo "exit=$rc $(date)" >> $O/steps.log
cat $O/prof_*_summary.log | tail -30
grep -h '^{' $O/bench_*.log | cut -c1-200
cat $O/steps.log
exit $rc
