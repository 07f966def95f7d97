#!/bin/bash
# HighWay layer with the relu sign mask in place of S: tests, HGCN step, kernel stats
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s29
mkdir -p "$O"
cd "$R"
step() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -o '"ms_per_step": [0-9.]*' "$O/$name.log" | head -1; tail -2 "$O/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step tests 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_sliced.py tests/test_gpu_parity.py tests/test_gpu_dist_ea.py tests/test_gpu_scale_cfg4.py -k "highway or HighWay or hgcn or HGCN or sliced or dropin or train"
step hgcn 300 python -u tools/dist_step.py --model HGCN --steps 21 --warmup 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof_hgcn" -o run --output-format csv \
  -- python3 "$R/tools/dist_step.py" --model HGCN --steps 5 --warmup 2 --attribute 0 > "$O/prof_hgcn.log" 2>&1 || exit $?
python3 "$R/tools/kstats.py" "$O/prof_hgcn/run_kernel_stats.csv" | head -12
echo done
