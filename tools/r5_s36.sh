#!/bin/bash
# weight + bias gradients from one product (ones column): tests, HGCN / GCN / GAT cfg-4 steps, HGCN kernel stats
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s36
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_act.py tests/test_gpu_parity.py tests/test_gpu_scale_cfg4.py tests/test_gpu_scale_dbp15k.py tests/test_gpu_dist_ea.py tests/test_gpu_sliced.py tests/test_gpu_gemm_range.py > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
timeout -k 10 300 python -u tools/dbg/ab_step.py --off tadb --model HGCN --steps 15 --warmup 3 > "$O/hgcn_off.log" 2>&1 || { tail -5 "$O/hgcn_off.log"; exit 1; }
grep -o '"ms_per_step": [0-9.]*' "$O/hgcn_off.log" | head -1
timeout -k 10 300 python -u tools/dist_step.py --model HGCN --steps 15 --warmup 3 > "$O/hgcn.log" 2>&1 || { tail -5 "$O/hgcn.log"; exit 1; }
grep -o '"ms_per_step": [0-9.]*' "$O/hgcn.log" | head -1
timeout -k 10 300 python -u tools/dbg/ab_step.py --off tadb --model GAT --steps 15 --warmup 3 > "$O/gat4_off.log" 2>&1 || { tail -5 "$O/gat4_off.log"; exit 1; }
grep -o '"ms_per_step": [0-9.]*' "$O/gat4_off.log" | head -1
timeout -k 10 300 python -u tools/dist_step.py --model GAT --steps 15 --warmup 3 > "$O/gat4.log" 2>&1 || { tail -5 "$O/gat4.log"; exit 1; }
grep -o '"ms_per_step": [0-9.]*' "$O/gat4.log" | head -1
timeout -k 10 300 python -u tools/dbg/ab_step.py --off tadb --model GCN --steps 15 --warmup 3 > "$O/gcn4_off.log" 2>&1 || { tail -5 "$O/gcn4_off.log"; exit 1; }
grep -o '"ms_per_step": [0-9.]*' "$O/gcn4_off.log" | head -1
timeout -k 10 300 python -u tools/dist_step.py --model GCN --steps 15 --warmup 3 > "$O/gcn4.log" 2>&1 || { tail -5 "$O/gcn4.log"; exit 1; }
grep -o '"ms_per_step": [0-9.]*' "$O/gcn4.log" | head -1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof_hgcn" -o run --output-format csv \
  -- python3 "$R/tools/dist_step.py" --model HGCN --steps 5 --warmup 2 --attribute 0 > "$O/prof_hgcn.log" 2>&1 || exit $?
python3 "$R/tools/kstats.py" "$O/prof_hgcn/run_kernel_stats.csv" | head -16
