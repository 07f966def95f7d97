#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s2
mkdir -p "$O"
cd "$R"
step() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "$O/$name.log"
  return $rc
}
step dist_ea 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_dist_ea.py tests/test_gpu_l1.py
rc=$?; case $rc in 124|137|134|139) exit $rc ;; esac
step rehearse4 600 python -u bench.py --gpus 4 --rehearse --entities 100000 --steps 3 --warmup 1 \
  --no-side --no-sinkhorn --no-train || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv \
  -- python3 "$R/tools/sk_one.py" 15000 3 100 > "$O/prof.log" 2>&1 || exit $?
echo done
