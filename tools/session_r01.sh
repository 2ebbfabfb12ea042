set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python tools/ab_kernels.py --rounds 5 --variants 1,0 > $O/ab.log 2>&1 && \
timeout -k 10 300 python bench.py --config mixed --steps 20 > $O/bench_mixed.log 2>&1 && \
timeout -k 10 400 python bench.py --config tcp64k --steps 10 > $O/bench_tcp64k.log 2>&1 && \
TAG=r01 AB_ARGS="--rounds 2 --variants 0 --cases udp1500_frames" bash tools/gpu_check.sh
