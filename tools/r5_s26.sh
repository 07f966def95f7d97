#!/bin/bash
# f16x2 ring: chunk size x waves per workgroup A/B; range tests on the default build
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s26
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_gemm_range.py > "$O/range.log" 2>&1 || { tail -20 "$O/range.log"; exit 1; }
tail -1 "$O/range.log"
timeout -k 10 900 python -u tools/dbg/gemm_ab.py libgnnea_nowpf.so libgnnea.so libgnnea_f58.so libgnnea_nowpf.so libgnnea.so libgnnea_f58.so > "$O/ab.log" 2>&1 || exit 1
grep "^{" "$O/ab.log" | cut -c1-260
