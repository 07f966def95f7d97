#!/bin/bash
# A/B of the GAT row-major passes at cfg-5 (bf16): old kernels (GNNEA_GAT_HG=0) vs the
# head-grouped pipelined ones (F = 4 / 8), GAT-EA step medians; then the GAT GPU tests.
set -u
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out
mkdir -p $OUT
for cfg in "0 4" "1 4" "1 8"; do
  set -- $cfg
  GNNEA_GAT_HG=$1 GNNEA_GAT_HG_F=$2 timeout -k 10 180 python tools/dist_step.py --model GAT \
    --dtype bf16 --entities 2000000 --steps 21 --warmup 3 > $OUT/gat_ab_$1_$2.log 2>&1 || exit $?
  echo "hg=$1 F=$2: $(tail -1 $OUT/gat_ab_$1_$2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_min_max"])')"
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "gat or GAT or bf16" > $OUT/gat_tests.log 2>&1
rc=$?; tail -3 $OUT/gat_tests.log; exit $rc
