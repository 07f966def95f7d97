#!/bin/bash
# default bench line + rocprof evidence (round_gpu_bench.sh), Sinkhorn PMC passes
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/round_gpu_bench.sh || exit $?
bash tools/sk_pmc15k.sh "$R/gpurun_out/skpmc_r5" || exit $?
echo done
