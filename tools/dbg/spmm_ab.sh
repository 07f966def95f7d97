#!/bin/bash
# A/B of the headline sliced SpMM: GNNEA_SPMM_PIPE=0 (one batch at a time) vs the pipelined
# default, bench headline only; then the sliced / SpMM GPU tests.
set -u
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out
mkdir -p $OUT
for p in 0 1 0 1; do
  GNNEA_SPMM_PIPE=$p timeout -k 10 200 python bench.py --headline-only --no-sinkhorn \
    --no-cpu-baseline --no-train > $OUT/spmm_ab_$p.log 2>&1 || exit $?
  echo "pipe=$p $(tail -1 $OUT/spmm_ab_$p.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"])')"
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "spmm or sliced or highway or gcn or GCN or hgcn" > $OUT/spmm_tests.log 2>&1
rc=$?; tail -3 $OUT/spmm_tests.log; exit $rc
