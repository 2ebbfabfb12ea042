#!/bin/bash
# One GPU session: parity tests, kernel A/B, bench, rocprofv3 kernel trace and
# two PMC passes (FETCH_SIZE, WRITE_SIZE — each in its own run, no tracing
# domains besides the kernel trace).  Every GPU step has its own time limit;
# steps are chained with && so the first failure (or timeout) ends the session.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${TAG:-r01}
mkdir -p $O
cd $R
BENCH_PROF="--steps 10 --warmup 2 --no-cpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python tools/ab_kernels.py ${AB_ARGS:-} > $O/ab.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 12 > $O/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --config mixed --steps 20 --no-cpu > $O/bench_mixed.log 2>&1 && \
timeout -k 10 300 python bench.py --config fill --steps 20 --no-cpu > $O/bench_fill.log 2>&1 && \
timeout -k 10 400 python bench.py --config tcp64k --steps 10 --no-cpu > $O/bench_tcp64k.log 2>&1 && \
timeout -k 10 300 python bench.py --config e2e --steps 5 --no-cpu > $O/bench_e2e.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_trace -o run --output-format csv -- python3 $R/bench.py $BENCH_PROF > $O/prof_trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/prof_fetch -o run --output-format csv -- python3 $R/bench.py $BENCH_PROF > $O/prof_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/prof_write -o run --output-format csv -- python3 $R/bench.py $BENCH_PROF > $O/prof_write.log 2>&1 && \
cd $R && python tools/pmc_summary.py --fetch $O/prof_fetch --write $O/prof_write --trace $O/prof_trace \
    --probe-bytes 1572864000 --alg-bytes $((1048576 * 1516 + 524288)) --label "$TAG bench.py udp1500 frames" \
    --out $O/${TAG}_pmc_udp1500.json > $O/pmc_summary.log 2>&1
echo "exit=$?" >> $O/steps.log
