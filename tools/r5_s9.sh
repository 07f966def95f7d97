#!/bin/bash
# Whole -m gpu suite on the pruned library (-rA: the recorded GAT gradient errors), smoke, then the
# Sinkhorn rate, the cfg-5 cast trace and the HGCN step profile.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s9
mkdir -p "$O"
cd "$R"
step() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
step gpu_all 600 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread \
  -p no:cacheprovider
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step sk_rate 200 python -c "
import json, torch, bench
r = bench.sinkhorn_large(torch.device('cuda', 0))
print(json.dumps(r))"
step casts 200 python -u tools/dbg/cast_trace.py 20000
step hgcn_step 300 python -u tools/dist_step.py --model HGCN --steps 21 --warmup 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_hgcn" -o run --output-format csv \
  -- python3 "$R/tools/dist_step.py" --model HGCN --steps 5 --warmup 3 > "$O/prof_hgcn.log" 2>&1 || exit $?
echo done
