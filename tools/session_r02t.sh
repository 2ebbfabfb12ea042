#!/bin/bash
# SQ/GRBM counters: where the flat kernel's cycles go, mixed vs udp1500
set -o pipefail
mkdir -p gpurun_out/sq
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for c in mixed udp1500; do
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -d $R/gpurun_out/sq/$c -o run --output-format csv -- python3 $R/bench.py --config $c --steps 10 --warmup 2 --no-cpu > $R/gpurun_out/sq/$c.log 2>&1 || { tail -5 $R/gpurun_out/sq/$c.log; exit 1; }
done
cd $R && python3 tools/sq_summary.py gpurun_out/sq/mixed && python3 tools/sq_summary.py gpurun_out/sq/udp1500
