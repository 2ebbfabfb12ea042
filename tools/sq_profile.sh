#!/bin/bash
# SQ counter passes (each its own rocprofv3 run, kernel trace only) over the
# A/B tool on the given cases/variants.  Usage: CASES=... VARIANTS=... bash tools/sq_profile.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/sq
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $O/counters_list.txt 2>&1 || true
ARGS="--rounds 1 --reps 2 --variants ${VARIANTS:-0} --cases ${CASES:-udp1500_frames,cfg3_zipf_frames}"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS -d $O/p1 -o run --output-format csv -- python3 $R/tools/ab_kernels.py $ARGS > $O/p1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/p2 -o run --output-format csv -- python3 $R/tools/ab_kernels.py $ARGS > $O/p2.log 2>&1
echo "exit=$?" > $O/done.txt
