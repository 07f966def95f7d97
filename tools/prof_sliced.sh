#!/bin/bash
# rocprofv3 evidence for the bench's SpMM: kernel-trace stats of the bench, then FETCH_SIZE and
# WRITE_SIZE in passes of their own; summary -> gpurun_out/spmm_pmc.json.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out
K=${1:-k_spmm_sliced}
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof_b" -o run --output-format csv \
  -- python "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-train > "$O/prof_b.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$O/pmc_f" -o run --output-format csv \
  -- python "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-sinkhorn --no-train > "$O/pmc_f.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$O/pmc_w" -o run --output-format csv \
  -- python "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-sinkhorn --no-train > "$O/pmc_w.log" 2>&1 || exit $?
python "$R/tools/pmc_summary.py" $(find "$O/pmc_f" -name "*counter_collection.csv" | head -1) \
  $(find "$O/pmc_w" -name "*counter_collection.csv" | head -1) "$K" "$O/spmm_pmc.json"
