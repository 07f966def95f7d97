set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
GNNEA_BF16W_RING=1 timeout -k 10 400 $T -x tests/test_gpu_bf16.py -k "gemm" > gpurun_out/t_gemm.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" gpurun_out/t_gemm.log | head -30; tail -5 gpurun_out/t_gemm.log; exit 1; }
tail -1 gpurun_out/t_gemm.log
for v in 0 1 0 1; do GNNEA_BF16W_RING=$v timeout -k 10 120 python tools/dbg/bf16w_ab.py || exit 1; done
bash tools/gpu_round.sh tests smoke bench hgcn gat4 gat5
