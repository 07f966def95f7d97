#!/bin/bash
# Sinkhorn GPU session: the fused / timeout / fixture tests, the B = 15000 rates, a kernel trace.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/sk
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_sinkhorn_fused.py tests/test_gpu_sinkhorn_timeout.py tests/test_gpu_parity.py -k "sinkhorn or gw or fused or timeout or knopp" \
  > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -3 "$O/tests.log"
timeout -k 10 300 python -c "
import json, torch, bench
r = bench.sinkhorn_large(torch.device('cuda', 0))
print(json.dumps(r))" > "$O/rate15k.json" 2> "$O/rate15k.err" || { tail "$O/rate15k.err"; exit 1; }
cat "$O/rate15k.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv \
  -- python3 "$R/tools/sk_one.py" 15000 3 100 > "$O/prof.log" 2>&1 || exit $?
echo done
