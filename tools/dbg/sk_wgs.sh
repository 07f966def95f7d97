#!/bin/bash
# Sinkhorn iters/s at B = 3000 for several sweep workgroup counts (GNNEA_SK_WGS)
cd "$(dirname "$0")/../.."
for w in 128 192 256 384 512; do
  GNNEA_SK_WGS=$w timeout -k 10 120 python -c "
import sys, torch; sys.path.insert(0,'gnn-mtl_amd'); sys.path.insert(0,'.')
import bench
print($w, bench.sinkhorn_rate(torch.device('cuda:0'))['iters_per_s'], flush=True)
" || exit $?
done
