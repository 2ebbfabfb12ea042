set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_rows2.log 2>&1 || { tail -30 gpurun_out/t_rows2.log; exit 1; }
tail -1 gpurun_out/t_rows2.log
timeout -k 10 600 python -u tools/ab_kernels.py --rounds 6 --variants 0,2,1 --cases udp1500_slots > gpurun_out/ab_rows2.log 2>&1 || { tail -20 gpurun_out/ab_rows2.log; exit 1; }
grep case gpurun_out/ab_rows2.log
timeout -k 10 300 python -u bench.py --config e2e --steps 5 --no-cpu > gpurun_out/b_e2e2.log 2>&1 || { tail -20 gpurun_out/b_e2e2.log; exit 1; }
grep -o '"A_slots_as_is": {[^}]*}' gpurun_out/b_e2e2.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -2 gpurun_out/smoke.log
