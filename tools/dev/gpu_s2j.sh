set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_sparse.log 2>&1 || { tail -30 gpurun_out/t_sparse.log; exit 1; }
tail -1 gpurun_out/t_sparse.log
V="0,16,16:::::::::0,1"
timeout -k 10 600 python -u tools/ab_kernels.py --rounds 8 --variants $V --cases udp1500_slots > gpurun_out/ab_slots2.log 2>&1 || { tail -20 gpurun_out/ab_slots2.log; exit 1; }
grep case gpurun_out/ab_slots2.log
timeout -k 10 300 python -u bench.py --config e2e --steps 5 --no-cpu > gpurun_out/b_e2e.log 2>&1 || { tail -20 gpurun_out/b_e2e.log; exit 1; }
grep -o '"variants": .*' gpurun_out/b_e2e.log | cut -c1-400
