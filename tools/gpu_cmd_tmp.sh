bash tools/round_gpu_tests.sh
