#!/bin/bash
# dW (k_gemm_ta_x3d): A splits interleaved with the first B fragment's MFMAs vs not
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s28
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_gpu_gemm_range.py -k "layer or gemm or x3 or range" > "$O/tests.log" 2>&1 || { tail -20 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
timeout -k 10 600 python -u tools/dbg/gemm_ab.py libgnnea_noilv.so libgnnea.so libgnnea_noilv.so libgnnea.so > "$O/ab.log" 2>&1 || exit 1
grep "^{" "$O/ab.log" | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); k = next(iter(d)); v = d[k]
    print(k, {x: v[x] for x in v if 'dW' in x})"
timeout -k 10 300 python -u tools/dist_step.py --model HGCN --steps 15 --warmup 3 --attribute 0 > "$O/hgcn.log" 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' "$O/hgcn.log" | head -1
