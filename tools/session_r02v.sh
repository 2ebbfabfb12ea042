#!/bin/bash
# transposed-scan forms (24-26): parity on the variant tests, then A/B
set -o pipefail
mkdir -p gpurun_out
python - <<'PY' > /dev/null
PY
timeout -k 10 600 python -u tools/ab_kernels.py --rounds 6 --reps 5 --rotate 4 \
  --cases udp1500x2_frames,udp1500_frames,cfg3_zipf_frames,zipf_spans,tcp64k_spans \
  --variants 16,26,15,25 > gpurun_out/ab_tscan.log 2>&1 || { tail -20 gpurun_out/ab_tscan.log; exit 1; }
cat gpurun_out/ab_tscan.log
