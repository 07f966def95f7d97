set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale_dbp15k.py tests/test_gpu_parity.py tests/test_gpu_sinkhorn_shard.py tests/test_gpu_l1.py -x -q -k "sinkhorn or gw or fgw or wasser or uea or ot" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/sk_tests.log 2>&1; rc=$?; tail -3 gpurun_out/sk_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "
import sys, json; sys.argv=['bench.py']
sys.path.insert(0, '.')
import torch, bench
d = torch.device('cuda:0')
print(json.dumps(bench.sinkhorn_rate(d)))
" 2>&1 | grep -v amdgpu.ids
