#!/bin/bash
# HighWay tail (gate recomputed, epilogue operands prefetched) + Sinkhorn 16-wave sweep
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s8
mkdir -p "$O"
cd "$R"
step() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
step hw_tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_sliced.py tests/test_gpu_scale_cfg4.py -k "highway or hgcn or HighWay or sliced"
bash tools/r5_sk.sh s8/sk || exit $?
step casts 300 python -u tools/dbg/cast_trace.py 20000
step hgcn_step 600 python -u tools/dist_step.py --model HGCN --steps 21 --warmup 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof_hgcn" -o run --output-format csv \
  -- python3 "$R/tools/dist_step.py" --model HGCN --steps 5 --warmup 3 > "$O/prof_hgcn.log" 2>&1 || exit $?
python3 "$R/tools/kstats.py" "$O/prof_hgcn/run_kernel_stats.csv" 2>/dev/null | head -20 || true
echo done
