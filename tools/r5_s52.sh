#!/bin/bash
# the four EA training steps on the final tree (one box): HGCN / GCN / GAT cfg-4, GAT cfg-5 bf16
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s52
mkdir -p "$O"
cd "$R"
run() {  # name args...
  local n=$1; shift
  timeout -k 10 400 python -u tools/dist_step.py "$@" --steps 21 --warmup 3 > "$O/$n.log" 2>&1 || { tail -5 "$O/$n.log"; exit 1; }
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' "$O/$n.log" | head -1)"
}
run hgcn --model HGCN
run gcn --model GCN
run gat4 --model GAT
run gat5 --model GAT --dtype bf16 --entities 2000000
