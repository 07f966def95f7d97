#!/bin/bash
# rocprofv3 evidence for the bench's SpMM: kernel-trace stats of the full bench, then PMC
# counters of the headline aggregation in passes of their own (each within the per-block limits:
# FETCH_SIZE uses 3 TCC counters, WRITE_SIZE 2); summary -> gpurun_out/spmm_pmc.json.
#   bash tools/prof_sliced.sh [kernel substring]
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out
K=${1:-k_spmm_sliced}
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof_b" -o run --output-format csv \
  -- python "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-train > "$O/prof_b.log" 2>&1 || exit $?
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_32B_sum"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $pmc -d "$O/pmc_$i" -o run --output-format csv \
    -- python "$R/bench.py" --steps 3 --warmup 1 --headline-only > "$O/pmc_$i.log" 2>&1 || exit $?
done
python "$R/tools/pmc_summary.py" "$K" "$O/spmm_pmc.json" \
  $(find "$O"/pmc_1 "$O"/pmc_2 "$O"/pmc_3 -name "*counter_collection.csv")
