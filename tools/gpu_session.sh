#!/bin/bash
# One parametrised GPU session (replaces round 2's one-off runners, which are in
# git history): run on the GPU box through gpurun, e.g.
#   gpurun --timeout 1200 -- 'bash tools/gpu_session.sh r03a pytest bench:udp1500 prof:fill'
# Steps (in order; each GPU step has its own time limit and the steps chain:
# the first failure, time limit or fault ends the session):
#   pytest                 the GPU test suite (-m gpu), one process
#   smoke                  __graft_entry__.smoke()
#   headline               bench.py as the driver runs it (N=1, CPU baseline included)
#   bench:CFG[+ARG...]     bench.py --config CFG --steps 20 --no-cpu ARG...   (ARGs joined by '+')
#   trace:CFG[+ARG...]     rocprofv3 --kernel-trace --stats of the bench command
#   prof:CFG[+ARG...]      trace + separate FETCH_SIZE and WRITE_SIZE passes of the bench command,
#                          cut to the timed dispatches by tools/prof_timed.py ($TAG_pmc_CFG.json)
#   sq:CFG[+ARG...]        two SQ counter passes of the bench command (instruction mix, waits; tools/pmc_sum.py)
#   py:SCRIPT[+ARG...]     python SCRIPT ARG... (a tools/ probe)
#   bin:PROGRAM[+ARG...]   a probe program built here beforehand (tools/dev/*.hip)
#   pbin:PROGRAM[+ARG...]  the same program under rocprofv3: a kernel trace, then separate FETCH_SIZE and
#                          WRITE_SIZE passes; per-kernel means by tools/pmc_by_name.py (pbin_NAME_summary.log)
#   lib:PATH | lib:default the library later steps load (SCCSUM_LIB: an A/B build of the same ABI,
#                          or libsccsum_at_<commit>.so, an older tree's build); bench logs are named after it
# Outputs go to gpurun_out/TAG/; steps.log records each step's outcome.
set -o pipefail
TAG=${1:?usage: gpu_session.sh TAG STEP...}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R" || exit 1
export TMPDIR=/tmp
PROF_STEPS="--steps 10 --warmup 2 --no-cpu"
LIBTAG=

split() {  # split CFG+A+B -> CFG and args array ARGS
    local IFS='+'
    read -r -a parts <<< "$1"
    CFG=${parts[0]}
    ARGS=("${parts[@]:1}")
}

name_of() {  # file-name form of a step's config + args
    echo "$1" | tr '+/' '__' | tr -d '-'
}

run_step() {
    local step=$1 kind=${1%%:*} rest=${1#*:}
    local n
    n=$(name_of "$rest")
    case $kind in
        pytest)
            timeout -k 10 900 python -u -m pytest tests -m gpu ${PYTEST_X--x} -v --timeout 120 --timeout-method thread \
                > "$O/pytest_gpu.log" 2>&1 ;;
        smoke)
            timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > "$O/smoke.log" 2>&1 ;;
        headline)
            timeout -k 10 400 python bench.py > "$O/bench_headline.log" 2>&1 ;;
        bench)
            split "$rest"
            timeout -k 10 400 python bench.py --config "$CFG" --steps 20 --no-cpu "${ARGS[@]}" \
                >> "$O/bench_$n$LIBTAG.log" 2>&1 ;;
        lib)
            if [ "$rest" = default ]; then
                unset SCCSUM_LIB SCCSUM_ABI_ANY
                LIBTAG=
            else
                export SCCSUM_LIB=$R/$rest
                LIBTAG=_$(basename "$rest" .so)
                # libsccsum_at_<commit>.so: an older tree's build (maybe another ABI version)
                case $rest in *libsccsum_at_*) export SCCSUM_ABI_ANY=1 ;; *) unset SCCSUM_ABI_ANY ;; esac
            fi ;;
        trace)
            split "$rest"
            (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace_$n" -o run \
                --output-format csv -- python3 "$R/bench.py" --config "$CFG" $PROF_STEPS "${ARGS[@]}") \
                > "$O/trace_$n.log" 2>&1 ;;
        prof)
            split "$rest"
            (cd /tmp && \
             timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$n/trace" -o run --output-format csv \
                -- python3 "$R/bench.py" --config "$CFG" $PROF_STEPS "${ARGS[@]}" > "$O/prof_${n}_trace.log" 2>&1 && \
             timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$O/prof_$n/fetch" -o run --output-format csv \
                -- python3 "$R/bench.py" --config "$CFG" $PROF_STEPS "${ARGS[@]}" > "$O/prof_${n}_fetch.log" 2>&1 && \
             timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$O/prof_$n/write" -o run --output-format csv \
                -- python3 "$R/bench.py" --config "$CFG" $PROF_STEPS "${ARGS[@]}" > "$O/prof_${n}_write.log" 2>&1) && \
            python tools/prof_timed.py --bench-log "$O/prof_${n}_trace.log" --trace "$O/prof_$n/trace" \
                --fetch "$O/prof_$n/fetch" --write "$O/prof_$n/write" --probe-bytes "${PROBE_BYTES:-0}" \
                --config "$CFG" --label "$TAG bench.py --config $CFG $PROF_STEPS ${ARGS[*]}" \
                --out "$O/${TAG}_pmc_$n.json" --trace-out "$O/${TAG}_trace_$n.csv" > "$O/prof_${n}_summary.log" 2>&1 ;;
        sq)  # two SQ counter passes of the bench command (instruction mix, wait cycles), summed per kernel
            split "$rest"
            (cd /tmp && \
             timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM \
                SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d "$O/sq_$n/a" -o run \
                --output-format csv -- python3 "$R/bench.py" --config "$CFG" $PROF_STEPS "${ARGS[@]}" \
                > "$O/sq_${n}_a.log" 2>&1 && \
             timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_VALU \
                SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH -d "$O/sq_$n/b" -o run \
                --output-format csv -- python3 "$R/bench.py" --config "$CFG" $PROF_STEPS "${ARGS[@]}" \
                > "$O/sq_${n}_b.log" 2>&1) && \
            python tools/pmc_sum.py "$O/sq_$n/a" "$O/sq_$n/b" > "$O/sq_${n}_summary.log" 2>&1 ;;
        py)
            split "$rest"
            timeout -k 10 400 python "$CFG" "${ARGS[@]}" >> "$O/py_$(basename "$CFG" .py).log" 2>&1 ;;
        bin)
            split "$rest"
            timeout -k 10 400 "./$CFG" "${ARGS[@]}" >> "$O/bin_$(basename "$CFG").log" 2>&1 ;;
        pbin)
            split "$rest"
            (cd /tmp && \
             timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/pbin_$n/trace" -o run --output-format csv \
                -- "$R/$CFG" "${ARGS[@]}" > "$O/pbin_${n}_trace.log" 2>&1 && \
             timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$O/pbin_$n/fetch" -o run --output-format csv \
                -- "$R/$CFG" "${ARGS[@]}" > "$O/pbin_${n}_fetch.log" 2>&1 && \
             timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$O/pbin_$n/write" -o run --output-format csv \
                -- "$R/$CFG" "${ARGS[@]}" > "$O/pbin_${n}_write.log" 2>&1) && \
            { python tools/pmc_by_name.py "$O/pbin_$n/fetch" --trace "$O/pbin_$n/trace" && \
              python tools/pmc_by_name.py "$O/pbin_$n/write" --write; } > "$O/pbin_${n}_summary.log" 2>&1 ;;
        *)
            echo "unknown step $step" >> "$O/steps.log"
            return 2 ;;
    esac
}

echo "start $(date)" >> "$O/steps.log"
rc=0
for step in "$@"; do
    run_step "$step"
    rc=$?
    echo "$step rc=$rc $(date +%T)" >> "$O/steps.log"
    [ $rc -eq 0 ] || break
done
echo "exit=$rc $(date)" >> "$O/steps.log"
grep -h '^{' "$O"/bench*.log 2>/dev/null | cut -c1-600
tail -3 "$O/pytest_gpu.log" 2>/dev/null
cat "$O/steps.log"
exit $rc
