#!/bin/bash
# Sinkhorn sweep: 64-entry exp table (degree-5 polynomial) vs 2048 (degree 3): tests + rate
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s21
mkdir -p "$O"
cd "$R"
step() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
GNNEA_LIB_FILE=libgnnea_tab64.so step tests64 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_sinkhorn_fused.py tests/test_gpu_sinkhorn_timeout.py tests/test_gpu_parity.py tests/test_gpu_scale_dbp15k.py -k "sinkhorn or gw or knopp or fused or timeout"
for lib in libgnnea.so libgnnea_tab64.so libgnnea.so libgnnea_tab64.so; do
  GNNEA_LIB_FILE=$lib step "sk_${lib%.so}" 200 python -c "
import json, torch, bench
r = bench.sinkhorn_large(torch.device('cuda', 0))
print(json.dumps({'lib': '$lib', 'rate': r['iters_per_s']}))"
done
echo done
