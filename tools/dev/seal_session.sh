set -o pipefail
O=gpurun_out/r06s1; mkdir -p $O
SCCSUM_FUZZ_SCALE=10 timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_fuzz.py tests/test_cpp_api.py tests/test_sharding.py -x -q --timeout 300 --timeout-method thread -k "engine or ring or shards or shard" > $O/engine_fuzz.log 2>&1 || { echo TESTS FAILED; exit 1; }
for i in 1 2; do
  timeout -k 10 120 ./tools/dev/engine_steps >> $O/steps_seal.log 2>&1 || exit 1
  LD_LIBRARY_PATH=$PWD/seastar_amd/lib/ab/prev3 timeout -k 10 120 ./tools/dev/engine_steps >> $O/steps_prev3.log 2>&1 || exit 1
done
ENGINE_STEPS_RING=65536 timeout -k 10 120 ./tools/dev/engine_steps >> $O/steps_seal_65536.log 2>&1 || exit 1
timeout -k 10 120 ./tools/dev/engine_steps producers 16 >> $O/steps_seal_producers16.log 2>&1 || exit 1
bash tools/gpu_session.sh r06s1 lib:default bench:mixed+--steps+100 lib:seastar_amd/lib/ab/libsccsum_prev3.so bench:mixed+--steps+100 lib:default bench:mixed+--steps+100 lib:seastar_amd/lib/ab/libsccsum_prev3.so bench:mixed+--steps+100 lib:default bench:udp1500+--launch+engine+--steps+200 lib:seastar_amd/lib/ab/libsccsum_prev3.so bench:udp1500+--launch+engine+--steps+200
