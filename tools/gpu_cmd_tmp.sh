set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_bf16.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/bf16_tests.log 2>&1 || { tail -30 gpurun_out/bf16_tests.log; exit 1; }
tail -1 gpurun_out/bf16_tests.log
timeout -k 10 120 python tools/gemm_bf16_bench.py > gpurun_out/gb1.json 2>&1 || { tail gpurun_out/gb1.json; exit 1; }
GNNEA_BF16_EPI=0 timeout -k 10 120 python tools/gemm_bf16_bench.py > gpurun_out/gb0.json 2>&1 || { tail gpurun_out/gb0.json; exit 1; }
tail -1 gpurun_out/gb1.json; tail -1 gpurun_out/gb0.json
