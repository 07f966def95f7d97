#!/bin/bash
# Sinkhorn check: the fused / timeout / fixture tests, the B = 15000 rate, a kernel trace.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/${1:-sk}
mkdir -p "$O"
cd "$R"
step() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
step sk_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_sinkhorn_fused.py tests/test_gpu_sinkhorn_timeout.py tests/test_gpu_parity.py \
  tests/test_gpu_scale_dbp15k.py -k "sinkhorn or gw or knopp or fused or timeout"
step sk_rate 300 python -c "
import json, torch, bench
r = bench.sinkhorn_large(torch.device('cuda', 0))
print(json.dumps(r))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv \
  -- python3 "$R/tools/sk_one.py" 15000 3 100 > "$O/prof.log" 2>&1 || exit $?
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/prof/run_kernel_stats.csv')))[:6]:
    print(r['Name'][:70], r['Calls'], r['AverageNs'])"
