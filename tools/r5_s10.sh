#!/bin/bash
# cfg-5 cast trace at the dispatcher (autograd-engine casts included)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s10
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u tools/dbg/cast_trace.py 200000 > "$O/casts.log" 2>&1
rc=$?; tail -30 "$O/casts.log" | cut -c1-400; exit $rc
