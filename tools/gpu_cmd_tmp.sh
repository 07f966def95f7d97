set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T -x tests/test_gpu_parity.py -k "onchip" > gpurun_out/t_skres.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" gpurun_out/t_skres.log | head -30; tail -5 gpurun_out/t_skres.log; exit 1; }
tail -1 gpurun_out/t_skres.log
timeout -k 10 200 python tools/sk_bench.py 3000 1000
timeout -k 10 400 $T -x tests/test_gpu_parity.py tests/test_gpu_scale_dbp15k.py -k "sinkhorn" > gpurun_out/t_sk.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" gpurun_out/t_sk.log | head -30; tail -5 gpurun_out/t_sk.log; exit 1; }
tail -1 gpurun_out/t_sk.log
