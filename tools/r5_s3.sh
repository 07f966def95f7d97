#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s3
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u tools/dbg/halo_ab_dbg.py 100000 > "$O/halo_dbg.log" 2>&1
rc=$?; echo "halo_dbg rc=$rc"; grep "^{" "$O/halo_dbg.log"
case $rc in 124|137|134|139) exit $rc ;; esac
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_dist_ea.py > "$O/dist_ea.log" 2>&1
echo "dist_ea rc=$?"; grep -o "AssertionError: .*" "$O/dist_ea.log" | cut -c1-600
