set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_slots.log 2>&1 || { tail -30 gpurun_out/t_slots.log; exit 1; }
tail -1 gpurun_out/t_slots.log
V="0,0:::::::::0,15,1"
timeout -k 10 600 python -u tools/ab_kernels.py --rounds 8 --variants $V --cases udp1500_slots,udp1500_frames,cfg3_zipf_frames,zipf_spans > gpurun_out/ab_slots.log 2>&1 || { tail -20 gpurun_out/ab_slots.log; exit 1; }
grep case gpurun_out/ab_slots.log
