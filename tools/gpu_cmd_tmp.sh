set -o pipefail
mkdir -p gpurun_out
bash tools/round_gpu_tests.sh || exit 1
timeout -k 10 400 python tools/dist_step.py --model GAT --entities 2000000 --dtype bf16 --steps 5 --warmup 1 > gpurun_out/step_gat_cfg5.json 2> gpurun_out/step_gat_cfg5.err || { tail -20 gpurun_out/step_gat_cfg5.err; exit 1; }
tail -1 gpurun_out/step_gat_cfg5.json | cut -c1-400
