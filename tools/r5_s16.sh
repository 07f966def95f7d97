#!/bin/bash
# GAT forward: first gather group issued before the row maximum; A/B on the cfg-5 / cfg-4 steps
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s16
mkdir -p "$O"
cd "$R"
step() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -o '"ms_per_step": [0-9.]*' "$O/$name.log" | head -1; tail -1 "$O/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_gpu_sliced.py tests/test_gpu_bf16.py -k "gat or GAT"
for lib in libgnnea_gatold.so libgnnea.so libgnnea_gatold.so libgnnea.so; do
  GNNEA_LIB_FILE=$lib step "gat5_${lib%.so}" 300 python -u tools/dist_step.py --model GAT --dtype bf16 --entities 2000000 --steps 15 --warmup 3 --attribute 0
done
for lib in libgnnea_gatold.so libgnnea.so; do
  GNNEA_LIB_FILE=$lib step "gat4_${lib%.so}" 300 python -u tools/dist_step.py --model GAT --steps 15 --warmup 3 --attribute 0
done
echo done
