#!/bin/bash
# GAT work loop: GAT / bf16 / colsum GPU tests, then the cfg-5 bf16 GAT-EA step under a
# rocprofv3 kernel trace (per-kernel times), then the cfg-4 fp32 GAT-EA step.
set -u
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "gat or GAT or bf16 or colsum ${EXTRA_K:-}" > $OUT/gat_tests.log 2>&1
rc=$?; tail -3 $OUT/gat_tests.log; [ $rc -eq 0 ] || exit $rc
for s in ${STEPS:-gat5 gat4}; do
  case $s in
    gat5) a="--model GAT --dtype bf16 --entities 2000000" ;;
    gat4) a="--model GAT" ;;
    hgcn) a="--model HGCN" ;;
  esac
  rm -rf $OUT/prof_$s
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$s" -o run \
      --output-format csv -- python "${GRAFT_REPO_ROOT:-$PWD}/tools/dist_step.py" $a --steps 21 --warmup 3 ) \
      > "$OUT/prof_$s.log" 2>&1 || exit $?
  grep -h "\"ms_per_step\"" $OUT/prof_$s.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["model"][:8], d["dtype"][:5], d["ms_per_step"], d["ms_min_max"])'
  python tools/kstats.py $OUT/prof_$s/run_kernel_stats.csv 14 24
done
