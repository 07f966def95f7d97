#!/bin/bash
# A/B of the GAT source pass's record reads (k_gat_bwd_src_hg RD: one LDS-DMA per edge row
# instead of a 64-row gather): the GAT GPU tests on the variant build, then rocprofv3 kernel
# stats of the cfg-5 bf16 GAT-EA step (tools/dist_step.py), base and variant alternating.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/src_rd
mkdir -p "$O"
cd "$R"
GNNEA_LIB_FILE=libgnnea_rd.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider -k "gat or GAT or cfg5 or attention" \
  > "$O/tests_rd.log" 2>&1 || { tail -30 "$O/tests_rd.log"; exit 1; }
tail -2 "$O/tests_rd.log"
cd /tmp && export TMPDIR=/tmp
for v in base rd base rd; do
  lib=libgnnea.so; [ $v = rd ] && lib=libgnnea_rd.so
  i=$((${i:-0}+1))
  GNNEA_LIB_FILE=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/p${i}_$v" -o run \
    --output-format csv -- python "$R/tools/dist_step.py" --model GAT --dtype bf16 \
    --entities 2000000 --steps 11 --warmup 2 > "$O/step_${i}_$v.log" 2>&1 || exit $?
  tail -1 "$O/step_${i}_$v.log" | head -c 300; echo
done
