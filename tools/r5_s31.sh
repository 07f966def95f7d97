#!/bin/bash
# f16x2 ring GEMM: the second half of the waves starts later (s_sleep), de-phasing the two waves of a SIMD: A/B
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s31
mkdir -p "$O"
cd "$R"
timeout -k 10 700 python -u tools/dbg/gemm_ab.py libgnnea.so libgnnea_dp8.so libgnnea_dp24.so libgnnea_dp63.so libgnnea.so libgnnea_dp8.so libgnnea_dp24.so libgnnea_dp63.so > "$O/ab.log" 2>&1 || { tail -20 "$O/ab.log"; exit 1; }
grep "^{" "$O/ab.log"
