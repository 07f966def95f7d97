#!/bin/bash
# round-5 session 1: Sinkhorn (fused sweep waits, timeout path), sharded search / EAModel
# rehearsal, the N = 4 bench rehearsal with halo_ab.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s1
mkdir -p "$O"
cd "$R"
step() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "$O/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step sk_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_sinkhorn_fused.py tests/test_gpu_sinkhorn_timeout.py
step sk_parity 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py -k "sinkhorn or gw or knopp"
step sk_rate 300 python -c "
import json, torch, bench
r = bench.sinkhorn_large(torch.device('cuda', 0))
print(json.dumps(r))"
step dist_ea 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_dist_ea.py tests/test_gpu_l1.py
step rehearse4 600 python -u bench.py --gpus 4 --rehearse --entities 100000 --steps 3 --warmup 1 \
  --no-side --no-sinkhorn --no-train
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv \
  -- python3 "$R/tools/sk_one.py" 15000 3 100 > "$O/prof.log" 2>&1 || exit $?
echo done
