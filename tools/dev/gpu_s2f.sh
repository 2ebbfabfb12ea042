set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_sc.log 2>&1 || { tail -30 gpurun_out/t_sc.log; exit 1; }
tail -1 gpurun_out/t_sc.log
V="0,0:::::::::0,0::::::::0"
timeout -k 10 500 python -u tools/ab_kernels.py --rounds 10 --variants $V --cases udp1500x2_frames,cfg3_zipf_frames,udp1500_frames,tcp64k_spans > gpurun_out/ab_sc.log 2>&1 || { tail -20 gpurun_out/ab_sc.log; exit 1; }
grep case gpurun_out/ab_sc.log
for a in "" "--config mixed" "--config mixed --launch single" "--config tcp64k --steps 10"; do
timeout -k 10 300 python -u bench.py --no-cpu $a > gpurun_out/b_sc.log 2>&1 || { tail -20 gpurun_out/b_sc.log; exit 1; }
echo "bench $a $(grep -o '"value": [0-9.]*\|"frac": [0-9.]*\|"avg_launch_us": [0-9.]*' gpurun_out/b_sc.log | tr '\n' ' ')"
done
