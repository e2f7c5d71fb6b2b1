V=$PWD/ldpc-neuralnetwork-decoder_amd/ldpc_neural_decoder/_lib/variants
LDPC_AMD_LIB=$V/zflag.so timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu -p no:cacheprovider tests/test_flood_gpu.py tests/test_harness_gpu.py > gpurun_out/zflag_tests.log 2>&1 || { tail -20 gpurun_out/zflag_tests.log; exit 1; }
tail -1 gpurun_out/zflag_tests.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gnn_gpu.py tests/test_gnn_et_gpu.py tests/test_gnn_depth_gpu.py > gpurun_out/bf16_tests.log 2>&1 || { tail -20 gpurun_out/bf16_tests.log; exit 1; }
tail -1 gpurun_out/bf16_tests.log
bash tools/gpu_ab_flood.sh || exit 1
REPS=1 CASES="bf16_new:gnn-z32-bf16-i10:X=1 bf16_old:gnn-z32-bf16-i10:LDPC_AMD_LIB=$V/relu_f32.so bf16et_new:gnn-z32-bf16:X=1" bash tools/gpu_ab_gnn.sh 0
