#!/bin/bash
# f16x2 pipe kernel: range test, A/B vs the ring kernel, HGCN step; cfg-5 cast trace
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s11
mkdir -p "$O"
cd "$R"
step() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-900
  [ $rc -eq 0 ] || exit $rc
}
step range 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_gemm_range.py
step ab 400 python -u tools/dbg/gemm_ab.py libgnnea.so libgnnea_ring.so libgnnea.so
step hgcn_step 300 python -u tools/dist_step.py --model HGCN --steps 21 --warmup 3
step casts 300 python -u tools/dbg/cast_trace.py 200000
echo done
