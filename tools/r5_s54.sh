#!/bin/bash
# GAT sliced bwd_dst: heads and a values read before the dz chain: tests, cfg-4 A/B
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s54
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_gpu_bf16.py tests/test_gpu_sliced.py tests/test_gpu_scale_cfg5.py -k "gat or GAT" > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
for v in old new old new; do
  if [ $v = old ]; then export GNNEA_LIB_FILE=libgnnea_olddsts.so; else unset GNNEA_LIB_FILE; fi
  timeout -k 10 400 python -u tools/dist_step.py --model GAT --steps 15 --warmup 3 --attribute 0 > "$O/gat4_$v.log" 2>&1 || { tail -5 "$O/gat4_$v.log"; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' "$O/gat4_$v.log" | head -1)"
done
unset GNNEA_LIB_FILE
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof_gat4" -o run --output-format csv \
  -- python3 "$R/tools/dist_step.py" --model GAT --steps 5 --warmup 2 --attribute 0 > "$O/prof_gat4.log" 2>&1 || exit $?
python3 "$R/tools/kstats.py" "$O/prof_gat4/run_kernel_stats.csv" | grep -i "dst\|kernel " 
