#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s5
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u tools/dbg/halo_bwd_dbg.py 100000 > "$O/dbg.log" 2>&1
rc=$?; echo "dbg rc=$rc"; grep "^{" "$O/dbg.log"; tail -3 "$O/dbg.log"
