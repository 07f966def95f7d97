set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_scale_cfg5.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/bf16_tests.log 2>&1 || { tail -30 gpurun_out/bf16_tests.log; exit 1; }
tail -1 gpurun_out/bf16_tests.log
timeout -k 10 200 python tools/gemm_bf16_bench.py > gpurun_out/gb1.json 2>&1 || { tail gpurun_out/gb1.json; exit 1; }
timeout -k 10 200 python tools/gemm_bf16_bench.py --rows 2000000 > gpurun_out/gb2.json 2>&1 || { tail gpurun_out/gb2.json; exit 1; }
tail -1 gpurun_out/gb1.json; tail -1 gpurun_out/gb2.json
timeout -k 10 400 python tools/dist_step.py --model GAT --entities 2000000 --dtype bf16 --steps 5 --warmup 1 > gpurun_out/step_gat_cfg5q.json 2> gpurun_out/step_gat_cfg5q.err || { tail -20 gpurun_out/step_gat_cfg5q.err; exit 1; }
tail -1 gpurun_out/step_gat_cfg5q.json | cut -c400-700
