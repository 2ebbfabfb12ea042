set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "verify_only or multi_batch or udp1500 or tail_split" > gpurun_out/t_vo.log 2>&1 || { tail -30 gpurun_out/t_vo.log; exit 1; }
tail -2 gpurun_out/t_vo.log
for a in "" "--rx-out2" "" "--rx-out2"; do
timeout -k 10 300 python -u bench.py --no-cpu $a > gpurun_out/b_vo.log 2>&1 || { tail -20 gpurun_out/b_vo.log; exit 1; }
echo "udp1500 $a $(grep -o '"value": [0-9.]*\|"frac": [0-9.]*\|"avg_launch_us": [0-9.]*' gpurun_out/b_vo.log | tr '\n' ' ')"
done
for a in "" "--rx-out2"; do
timeout -k 10 300 python -u bench.py --config mixed --no-cpu $a > gpurun_out/b_vo.log 2>&1 || { tail -20 gpurun_out/b_vo.log; exit 1; }
echo "mixed $a $(grep -o '"value": [0-9.]*\|"frac": [0-9.]*\|"avg_launch_us": [0-9.]*' gpurun_out/b_vo.log | tr '\n' ' ')"
done
