#!/bin/bash
# x3 GEMM N-tile width sweep at 2M rows (GNNEA_X3_WT tuning override)
set -e
for wt in 0 2 4; do
  if [ $wt = 0 ]; then unset GNNEA_X3_WT; else export GNNEA_X3_WT=$wt; fi
  echo "== wt=$wt"
  timeout -k 10 200 python tools/gemm_bench.py --rows 2000000 --reps 5 --out gpurun_out/gemm2m_wt$wt.json | cut -c1-120
done
