#!/bin/bash
# x3 GEMM N-tile width sweep at DBP15K rows (GNNEA_X3_WT tuning override)
set -e
for wt in 0 1 2 3 4; do
  if [ $wt = 0 ]; then unset GNNEA_X3_WT; else export GNNEA_X3_WT=$wt; fi
  echo "== wt=$wt"
  timeout -k 10 120 python tools/gemm_bench.py --rows 30000 --reps 20 --out gpurun_out/gemm_wt$wt.json | cut -c1-160
done
