set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 600 python tools/ab_kernels.py --rounds 6 --rotate 4 --variants 1,6,8,13,14,15,16 > $O/ab.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 12 > $O/bench.log 2>&1
