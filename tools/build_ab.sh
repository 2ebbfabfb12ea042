#!/bin/bash
# Build A/B variants of libsccsum.so (same sources and ABI, one -D switch each)
# into seastar_amd/lib/ab/, for tools/gpu_session.sh's lib:PATH step, e.g.
#   bash tools/build_ab.sh nt0=SCCSUM_SOME_SWITCH b=SWITCH_A,SWITCH_B=2
# builds seastar_amd/lib/ab/libsccsum_nt0.so (-DSCCSUM_SOME_SWITCH) and libsccsum_b.so.
set -e
cd "$(dirname "$0")/.."
mkdir -p seastar_amd/lib/ab
SRC="seastar_amd/csrc/sccsum.hip seastar_amd/csrc/checksummer.cc seastar_amd/csrc/pipeline.cc seastar_amd/csrc/burst.cc"
FL="-O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -Wall -Wno-unused-command-line-argument -I include ${AB_FLAGS--mllvm -amdgpu-atomic-optimizer-strategy=None}"  # (build.py's device flags unless AB_FLAGS is set)
pids=()
for spec in "$@"; do
    name=${spec%%=*}
    defs=${spec#*=}
    D=""
    IFS=',' read -r -a dl <<< "$defs"
    for d in "${dl[@]}"; do D="$D -D$d"; done
    /opt/rocm/bin/hipcc $FL $D $SRC -o "seastar_amd/lib/ab/libsccsum_$name.so" &
    pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
ls -l seastar_amd/lib/ab/
