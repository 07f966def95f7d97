#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s24
mkdir -p "$O"
cd "$R"
timeout -k 10 200 python -u tools/dbg/f2_stamps.py 600 > "$O/st600.log" 2>&1 || exit 1
timeout -k 10 200 python -u tools/dbg/f2_stamps.py 300 > "$O/st300.log" 2>&1 || exit 1
timeout -k 10 300 python -u tools/dbg/gemm_ab.py libgnnea_stamp.so libgnnea.so > "$O/ab.log" 2>&1 || exit 1
grep -v amdgpu.ids "$O/st600.log"; grep -v amdgpu.ids "$O/st300.log"; grep "^{" "$O/ab.log" | cut -c1-200
