#!/bin/bash
# f16x2 ring GEMM with two 16-row blocks per wave (each weight fragment pair feeds six MFMAs): A/B
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s30
mkdir -p "$O"
cd "$R"
timeout -k 10 700 python -u tools/dbg/gemm_ab.py libgnnea.so libgnnea_rb2a.so libgnnea_rb2b.so libgnnea_rb2c.so libgnnea.so libgnnea_rb2a.so libgnnea_rb2b.so > "$O/ab.log" 2>&1 || { tail -20 "$O/ab.log"; exit 1; }
grep "^{" "$O/ab.log"
