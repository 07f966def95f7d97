set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dist_layers.py tests/test_gpu_sinkhorn_shard.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/dist_gpu.log 2>&1 || { tail -30 gpurun_out/dist_gpu.log; exit 1; }
tail -2 gpurun_out/dist_gpu.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 4 --rehearse --entities 200000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rehearse4.log 2>&1 || { tail -30 gpurun_out/rehearse4.log; exit 1; }
tail -1 gpurun_out/rehearse4.log | cut -c1-300
