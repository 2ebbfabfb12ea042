set -o pipefail
mkdir -p gpurun_out
V="0,0::::::::1,0::::::::2,0::::::::3,0::::::::4"
timeout -k 10 500 python -u tools/ab_kernels.py --rounds 8 --variants $V --cases udp1500x2_frames,cfg3_zipf_frames,udp1500_frames > gpurun_out/ab_outpol.log 2>&1 || { tail -20 gpurun_out/ab_outpol.log; exit 1; }
grep case gpurun_out/ab_outpol.log
