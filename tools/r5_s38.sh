#!/bin/bash
# GCN-EA cfg-4 step kernel stats
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s38
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof_gcn" -o run --output-format csv \
  -- python3 "$R/tools/dist_step.py" --model GCN --steps 5 --warmup 2 --attribute 0 > "$O/prof_gcn.log" 2>&1 || exit $?
python3 "$R/tools/kstats.py" "$O/prof_gcn/run_kernel_stats.csv" | head -24
