#!/bin/bash
# bf16 margin loss kernels: tests, cfg-5 GAT-EA step
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s15
mkdir -p "$O"
cd "$R"
step() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
step tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_l1.py tests/test_gpu_bf16.py tests/test_gpu_scale_cfg5.py tests/test_gpu_dist_ea.py
step gat5 400 python -u tools/dist_step.py --model GAT --dtype bf16 --entities 2000000 --steps 21 --warmup 3
echo done
