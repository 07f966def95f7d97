#!/bin/bash
# the dbp15k EA step tests (GCN / GAT / HGCN) on the current tree, then the whole suite + smoke
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s55
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q -rA --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_scale_dbp15k.py > "$O/dbp.log" 2>&1 || { grep -E "^E |passed|failed" "$O/dbp.log" | head -20; exit 1; }
tail -1 "$O/dbp.log"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread \
  -p no:cacheprovider > "$O/gpu_all.log" 2>&1
rc=$?; tail -3 "$O/gpu_all.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit 1
tail -1 "$O/smoke.log"
