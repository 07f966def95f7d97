#!/bin/bash
# how MFMA-bound is the fp32 dW kernel: k_gemm_ta_x3d with 3 of its 6 products (timing only)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s41
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u tools/dbg/gemm_ab.py libgnnea.so libgnnea_half.so libgnnea.so libgnnea_half.so > "$O/ab.log" 2>&1 || { tail -20 "$O/ab.log"; exit 1; }
grep "^{" "$O/ab.log" | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); k = next(iter(d)); v = d[k]
    print(k, {x: v[x] for x in v if 'dW' in x})"
