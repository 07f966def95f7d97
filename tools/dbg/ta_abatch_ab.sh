#!/bin/bash
# A/B of k_gemm_ta_x3d's A-fragment reads (GNNEA_TA_ABATCH: all five issued at once after the
# step barrier, against one fragment ahead): the GEMM GPU tests on the variant, then
# tools/ta_bench.py on base and variant alternating.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/ta_ab
mkdir -p "$O"
cd "$R"
GNNEA_LIB_FILE=libgnnea_tab.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider -k "gemm or ta_ or grad" \
  > "$O/tests_tab.log" 2>&1 || { tail -30 "$O/tests_tab.log"; exit 1; }
tail -2 "$O/tests_tab.log"
for v in base tab base tab; do
  lib=libgnnea.so; [ $v = tab ] && lib=libgnnea_tab.so
  GNNEA_LIB_FILE=$lib timeout -k 10 200 python tools/ta_bench.py --reps 21 --out "$O/ta_$v.jsonl" \
    || exit $?
done
