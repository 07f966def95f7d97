#!/bin/bash
# Sinkhorn phased-exponential A/B + tests; cfg-5 GAT-EA and HGCN-EA step profiles
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s13
mkdir -p "$O"
cd "$R"
step() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
for lib in libgnnea_ph0.so libgnnea.so libgnnea_ph0.so libgnnea.so; do
  GNNEA_LIB_FILE=$lib step "sk_${lib%.so}" 200 python -c "
import json, torch, bench
r = bench.sinkhorn_large(torch.device('cuda', 0))
print(json.dumps({'lib': '$lib', 'rate': r['iters_per_s']}))"
done
step sk_tests 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_sinkhorn_fused.py tests/test_gpu_sinkhorn_timeout.py
step gat5 400 python -u tools/dist_step.py --model GAT --dtype bf16 --entities 2000000 --steps 21 --warmup 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof_gat5" -o run --output-format csv \
  -- python3 "$R/tools/dist_step.py" --model GAT --dtype bf16 --entities 2000000 --steps 5 --warmup 2 --attribute 0 > "$O/prof_gat5.log" 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof_hgcn" -o run --output-format csv \
  -- python3 "$R/tools/dist_step.py" --model HGCN --steps 5 --warmup 2 --attribute 0 > "$O/prof_hgcn.log" 2>&1 || exit $?
echo done
