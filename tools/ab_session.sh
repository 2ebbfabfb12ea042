# A/B session on the GPU box: parity tests, then tools/ab_kernels.py over $AB variants (rotated batches).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 600 python tools/ab_kernels.py --rounds 8 --cases udp1500_frames,cfg3_zipf_frames --rotate ${ROT:-4} --variants ${AB:-6,8,15,16} > $O/ab.log 2>&1
