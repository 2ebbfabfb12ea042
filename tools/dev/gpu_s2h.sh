set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "tile_orders or tile_shapes or tail_split" > gpurun_out/t_xcd.log 2>&1 || { tail -30 gpurun_out/t_xcd.log; exit 1; }
tail -1 gpurun_out/t_xcd.log
V="0,0::::2,0::::1"
timeout -k 10 500 python -u tools/ab_kernels.py --rounds 10 --variants $V --cases udp1500x2_frames,cfg3_zipf_frames,udp1500_frames,tcp64k_spans,zipf_spans > gpurun_out/ab_xcd.log 2>&1 || { tail -20 gpurun_out/ab_xcd.log; exit 1; }
grep case gpurun_out/ab_xcd.log
