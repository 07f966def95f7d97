#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s4
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u tools/dbg/rs_dbg.py 100000 300 > "$O/rs_dbg.log" 2>&1
rc=$?; echo "rs_dbg rc=$rc"; grep "^{" "$O/rs_dbg.log"; tail -3 "$O/rs_dbg.log"
case $rc in 124|137|134|139) exit $rc ;; esac
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_dist_ea.py > "$O/dist_ea.log" 2>&1
echo "dist_ea rc=$?"; tail -2 "$O/dist_ea.log"; grep -o "AssertionError: .*" "$O/dist_ea.log" | cut -c1-600
