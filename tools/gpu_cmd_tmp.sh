set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -v --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T -x tests/test_gpu_parity.py tests/test_gpu_bf16.py tests/test_gpu_sliced.py -k "gat or onchip or sinkhorn_family" > gpurun_out/t_gat.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" gpurun_out/t_gat.log | head -30; tail -5 gpurun_out/t_gat.log; exit 1; }
tail -1 gpurun_out/t_gat.log
timeout -k 10 300 python tools/dist_step.py --model GAT --entities 2000000 --dtype bf16 > gpurun_out/step_gat5.json 2> gpurun_out/step_gat5.err || { tail -5 gpurun_out/step_gat5.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/step_gat5.json')); print({k: d[k] for k in d if 'ms' in k})"
timeout -k 10 900 $T -x tests/test_gpu_scale_cfg5.py > gpurun_out/t_cfg5.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" gpurun_out/t_cfg5.log | head -30; tail -5 gpurun_out/t_cfg5.log; exit 1; }
tail -1 gpurun_out/t_cfg5.log
