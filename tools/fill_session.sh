#!/bin/bash
# GPU session for the in-place generate path: bench (fill + default), kernel
# trace and the two PMC passes on the fill bench, each step time-limited.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
P="--config fill --steps 10 --warmup 2 --no-cpu"
timeout -k 10 300 python bench.py --config fill --steps 20 --warmup 5 > $O/bench_fill.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_default.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/fill_trace -o run --output-format csv -- python3 $R/bench.py $P > $O/fill_trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/fill_fetch -o run --output-format csv -- python3 $R/bench.py $P > $O/fill_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/fill_write -o run --output-format csv -- python3 $R/bench.py $P > $O/fill_write.log 2>&1
echo "exit=$?" >> $O/fill_steps.log
