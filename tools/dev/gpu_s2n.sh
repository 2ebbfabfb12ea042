set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "fill" > gpurun_out/t_plan2.log 2>&1 || { tail -30 gpurun_out/t_plan2.log; exit 1; }
tail -1 gpurun_out/t_plan2.log
: > gpurun_out/ab_fill_plan2.log
for i in 1 2; do for f in 1 0; do
timeout -k 10 300 python -u bench.py --config fill --no-cpu --fill-plan $f > gpurun_out/b_plan.log 2>&1 || { tail -20 gpurun_out/b_plan.log; exit 1; }
echo "fill-plan $f $(grep -o '"value": [0-9.]*\|"frac": [0-9.]*\|"avg_launch_us": [0-9.]*' gpurun_out/b_plan.log | tr '\n' ' ')" | tee -a gpurun_out/ab_fill_plan2.log
done; done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_plan2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config fill --steps 10 --warmup 2 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/prof_plan2.log 2>&1
grep -i "fill_store\|csum_flat" $GRAFT_REPO_ROOT/gpurun_out/prof_plan2/run_kernel_stats.csv | cut -c1-60,170-260
