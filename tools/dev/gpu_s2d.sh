set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_nostore.log
for i in 1 2; do
for L in seastar_amd/lib/libsccsum.so seastar_amd/lib/libsccsum_tmp_nostore.so; do
echo "lib $L" >> gpurun_out/ab_nostore.log
SCCSUM_LIB=$L timeout -k 10 300 python -u tools/ab_kernels.py --rounds 8 --variants 0,0::::::::0 --cases udp1500x2_frames,cfg3_zipf_frames >> gpurun_out/ab_nostore.log 2>&1 || { tail -20 gpurun_out/ab_nostore.log; exit 1; }
done
done
grep "case\|lib" gpurun_out/ab_nostore.log
