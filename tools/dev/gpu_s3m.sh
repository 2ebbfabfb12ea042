#!/bin/bash
# PMC profiles of SURVEY §8(d)'s layout variants under their own keys
# (mixed_align64: cfg 3 (ii), frames on 64 B boundaries; tcp64k_seg65535: cfg 4
# with 65 535 B segments), then their bench lines reading them.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s3m
mkdir -p $O
cd $R
export TMPDIR=/tmp
STEPS_PROF="--steps 10 --warmup 2 --no-cpu"
prof() {  # prof <label> <config> <extra bench args...>
    local l=$1 c=$2; shift 2
    cd /tmp && \
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$l/trace -o run --output-format csv -- python3 $R/bench.py --config $c $STEPS_PROF "$@" > $O/prof_${l}_trace.log 2>&1 && \
    timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/prof_$l/fetch -o run --output-format csv -- python3 $R/bench.py --config $c $STEPS_PROF "$@" > $O/prof_${l}_fetch.log 2>&1 && \
    timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/prof_$l/write -o run --output-format csv -- python3 $R/bench.py --config $c $STEPS_PROF "$@" > $O/prof_${l}_write.log 2>&1 && \
    cd $R && python tools/prof_timed.py --bench-log $O/prof_${l}_trace.log --trace $O/prof_$l/trace \
        --fetch $O/prof_$l/fetch --write $O/prof_$l/write --probe-bytes 0 --config $l \
        --label "r02 bench.py --config $c $STEPS_PROF $*" \
        --out $O/r02_pmc_$l.json --trace-out $O/r02_trace_$l.csv > $O/prof_${l}_summary.log 2>&1
}
echo "start $(date)" > $O/steps.log
prof mixed_align64 mixed --align 64 && echo "prof align64 ok" >> $O/steps.log && \
prof tcp64k_seg65535 tcp64k --seg-len 65535 && echo "prof seg65535 ok" >> $O/steps.log && \
cp $O/r02_pmc_mixed_align64.json $O/r02_pmc_tcp64k_seg65535.json $R/profiles/ && \
timeout -k 10 300 python bench.py --config mixed --align 64 --steps 20 --no-cpu > $O/bench_mixed_align64.log 2>&1 && echo "align64 ok" >> $O/steps.log && \
timeout -k 10 400 python bench.py --config tcp64k --seg-len 65535 --steps 10 --no-cpu > $O/bench_tcp65535.log 2>&1 && echo "tcp65535 ok" >> $O/steps.log
rc=$?
echo "exit=$rc $(date)" >> $O/steps.log
grep -h "traffic_over_alg\|avg_us_timed\|frac_from_trace" $O/r02_pmc_*.json
grep -h '^{' $O/bench_*.log | cut -c1-160
cat $O/steps.log
exit $rc
