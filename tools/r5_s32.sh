#!/bin/bash
# cfg-5 bf16 GAT-EA step: timing and kernel stats after the bf16 margin loss
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s32
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u tools/dist_step.py --model GAT --dtype bf16 --entities 2000000 --steps 21 --warmup 3 > "$O/gat5.log" 2>&1 || { tail -5 "$O/gat5.log"; exit 1; }
grep -o '"ms_per_step": [0-9.]*' "$O/gat5.log" | head -1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof_gat5" -o run --output-format csv \
  -- python3 "$R/tools/dist_step.py" --model GAT --dtype bf16 --entities 2000000 --steps 5 --warmup 2 --attribute 0 > "$O/prof_gat5.log" 2>&1 || exit $?
python3 "$R/tools/kstats.py" "$O/prof_gat5/run_kernel_stats.csv" | head -30
