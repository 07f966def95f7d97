set -o pipefail
mkdir -p gpurun_out
rm -rf gpurun_out/prof_cfg5
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg5 -o run --output-format csv -- python tools/dist_step.py --model GAT --entities 2000000 --dtype bf16 --steps 3 --warmup 1 > gpurun_out/prof_cfg5.log 2>&1 || { tail -20 gpurun_out/prof_cfg5.log; exit 1; }
find gpurun_out/prof_cfg5 -name "*kernel_stats.csv"
