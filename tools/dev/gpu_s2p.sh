set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_chunk.log 2>&1 || { tail -30 gpurun_out/t_chunk.log; exit 1; }
tail -1 gpurun_out/t_chunk.log
timeout -k 10 600 python -u tools/ab_kernels.py --rounds 8 --variants 0,1 --cases udp1500_slots,udp1500_slots_verify > gpurun_out/ab_chunk.log 2>&1 || { tail -20 gpurun_out/ab_chunk.log; exit 1; }
grep case gpurun_out/ab_chunk.log
for c in slots frags; do
timeout -k 10 300 python -u bench.py --config $c --no-cpu > gpurun_out/b_chunk.log 2>&1 || { tail -20 gpurun_out/b_chunk.log; exit 1; }
echo "$c $(grep -o '"value": [0-9.]*\|"frac": [0-9.]*\|"avg_launch_us": [0-9.]*\|"GiBps_packet_bytes": [0-9.]*' gpurun_out/b_chunk.log | tr '\n' ' ')"
done
