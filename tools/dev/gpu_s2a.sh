set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "tail_split or tile_shapes or multi_batch" > gpurun_out/t_tail.log 2>&1 || { tail -30 gpurun_out/t_tail.log; exit 1; }
tail -2 gpurun_out/t_tail.log
V="0,0::::::2:4,0::::::4:4,0::::::8:4,0::::::4:8,0::::::4:2"
timeout -k 10 400 python -u tools/ab_kernels.py --rounds 8 --variants $V --cases udp1500x2_frames,udp1500_frames,cfg3_zipf_frames > gpurun_out/ab_tail.log 2>&1 || { tail -20 gpurun_out/ab_tail.log; exit 1; }
cat gpurun_out/ab_tail.log | grep case
timeout -k 10 300 python -u bench.py --config mixed --no-cpu > gpurun_out/b_mixed_multi.log 2>&1 || { tail -20 gpurun_out/b_mixed_multi.log; exit 1; }
timeout -k 10 300 python -u bench.py --config mixed --launch single --no-cpu > gpurun_out/b_mixed_single.log 2>&1 || { tail -20 gpurun_out/b_mixed_single.log; exit 1; }
grep -o '"value": [0-9.]*\|"frac": [0-9.]*\|"avg_launch_us": [0-9.]*' gpurun_out/b_mixed_*.log
