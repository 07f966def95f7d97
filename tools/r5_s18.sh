#!/bin/bash
# N = 4 rehearsal on one device (gloo, host-staged): halo_ab, staged path, sharded loss / search
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s18
mkdir -p "$O"
cd "$R"
timeout -k 10 1000 python -u bench.py --gpus 4 --rehearse --steps 5 --warmup 2 > "$O/rehearse4.log" 2>&1
rc=$?
grep -v "amdgpu.ids" "$O/rehearse4.log" | tail -6 | cut -c1-1500
exit $rc
