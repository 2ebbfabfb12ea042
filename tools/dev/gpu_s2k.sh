set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_rows.log 2>&1 || { tail -30 gpurun_out/t_rows.log; exit 1; }
tail -1 gpurun_out/t_rows.log
timeout -k 10 600 python -u tools/ab_kernels.py --rounds 8 --variants 1,2,0,2:4,2:6 --cases udp1500_slots > gpurun_out/ab_rows.log 2>&1 || { tail -20 gpurun_out/ab_rows.log; exit 1; }
timeout -k 10 600 python -u tools/ab_kernels.py --rounds 6 --variants 0,2,1 --cases udp1500_frames,zipf_spans,cfg3_zipf_frames >> gpurun_out/ab_rows.log 2>&1 || { tail -20 gpurun_out/ab_rows.log; exit 1; }
grep case gpurun_out/ab_rows.log
