#!/bin/bash
# round-end bench line + rocprofv3 evidence of the headline SpMM (tools/round_gpu_bench.sh) on the
# current tree; outputs under gpurun_out/s51
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s51
mkdir -p "$O"
cd "$R"
timeout -k 10 700 python bench.py > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" > "$O/bench_line.json"
cat "$O/bench_line.json" | cut -c1-600
bash tools/prof_sliced.sh > "$O/prof_sliced.log" 2>&1 || { tail -20 "$O/prof_sliced.log"; exit 1; }
cat gpurun_out/spmm_pmc.json | head -40
