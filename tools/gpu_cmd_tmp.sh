set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T -x tests/test_gpu_bf16.py > gpurun_out/t_bf16.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" gpurun_out/t_bf16.log | head -30; tail -5 gpurun_out/t_bf16.log; exit 1; }
tail -1 gpurun_out/t_bf16.log
for wr in 1 0; do GNNEA_BF16_WRES=$wr timeout -k 10 120 python tools/gemm_bf16_bench.py || exit 1; done
timeout -k 10 400 $T -x tests/test_gpu_parity.py -k "gat" > gpurun_out/t_gat.log 2>&1 || { grep -E "FAIL|Error|assert|Timeout" gpurun_out/t_gat.log | head -30; tail -5 gpurun_out/t_gat.log; exit 1; }
tail -1 gpurun_out/t_gat.log
timeout -k 10 300 python tools/dist_step.py --model GAT --entities 2000000 --dtype bf16 > gpurun_out/step_gat5.json 2> gpurun_out/step_gat5.err || { tail -5 gpurun_out/step_gat5.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/step_gat5.json')); print({k: d[k] for k in d if 'ms' in k})"
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_skres2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/sk_one.py 3000 0 1000 > $GRAFT_REPO_ROOT/gpurun_out/prof_skres2.log 2>&1
grep -c k_sk_res $GRAFT_REPO_ROOT/gpurun_out/prof_skres2/run_kernel_trace.csv
