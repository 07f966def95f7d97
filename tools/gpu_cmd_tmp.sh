set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/dbg/sk_shard_rate.py 2>&1 | grep -v amdgpu.ids
