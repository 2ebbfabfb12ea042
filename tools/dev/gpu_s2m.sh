set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/steps_ab.log
for c in mixed udp1500; do for st in 20 100 20 100; do
timeout -k 10 300 python -u bench.py --config $c --no-cpu --steps $st > gpurun_out/b_st.log 2>&1 || { tail -20 gpurun_out/b_st.log; exit 1; }
echo "$c steps $st $(grep -o '"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"avg_launch_us": [0-9.]*' gpurun_out/b_st.log | tr '\n' ' ')" | tee -a gpurun_out/steps_ab.log
done; done
