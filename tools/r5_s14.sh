#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s14
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u tools/dbg/cast_trace.py 2000000 > "$O/casts5.log" 2>&1
rc=$?; tail -30 "$O/casts5.log" | cut -c1-500; exit $rc
