#!/bin/bash
# GCN layer's relu sign bits (fp32 sliced): tests, GCN-EA step A/B (old: the same build keeping Y, tools/dbg/ab_step.py --off gcnbits)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s48
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_sliced.py tests/test_gpu_parity.py tests/test_gpu_scale_cfg4.py tests/test_gpu_dist_ea.py tests/test_gpu_scale_dbp15k.py -k "gcn or GCN or sliced or sign" > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
for v in old new old new; do
  if [ $v = old ]; then a="tools/dbg/ab_step.py --off gcnbits"; else a="tools/dist_step.py"; fi
  timeout -k 10 300 python -u $a --model GCN --steps 15 --warmup 3 --attribute 0 > "$O/gcn_$v.log" 2>&1 || { tail -5 "$O/gcn_$v.log"; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' "$O/gcn_$v.log" | head -1)"
done
