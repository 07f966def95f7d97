set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sinkhorn_shard.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/shard.log 2>&1; rc=$?; tail -25 gpurun_out/shard.log; exit $rc
