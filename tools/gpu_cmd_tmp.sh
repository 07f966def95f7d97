set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T -x tests/test_gpu_sliced.py tests/test_gpu_parity.py -k "gemm" > gpurun_out/t_gemm.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" gpurun_out/t_gemm.log | head -30; tail -5 gpurun_out/t_gemm.log; exit 1; }
tail -1 gpurun_out/t_gemm.log
for v in 0 2 0 2; do GNNEA_X3W=$v timeout -k 10 120 python tools/dbg/x3_ab.py libgnnea.so | sed "s/^/x3w=$v /" || exit 1; done
