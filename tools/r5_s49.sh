#!/bin/bash
# whole -m gpu suite (-rA) + smoke on the current tree
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s49
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread \
  -p no:cacheprovider > "$O/gpu_all.log" 2>&1
rc=$?; tail -3 "$O/gpu_all.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit 1
tail -1 "$O/smoke.log"
