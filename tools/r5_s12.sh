#!/bin/bash
# GEMM A/B: ring (old), ring + row-stream lockstep, pipe; FETCH_SIZE of the 600-wide projection
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s12
mkdir -p "$O"
cd "$R"
step() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "$O/$name.log" | cut -c1-700
  [ $rc -eq 0 ] || exit $rc
}
cd /tmp && export TMPDIR=/tmp
for lib in libgnnea_ring.so libgnnea_rsync.so; do
  for shp in proj600 dx; do
    GNNEA_LIB_FILE=$lib timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_${lib%.so}_$shp" -o run --output-format csv \
      -- python3 "$R/tools/dbg/gemm_one.py" $shp 3 > "$O/pmc_${lib%.so}_$shp.log" 2>&1 || exit 1
    python3 - "$O/pmc_${lib%.so}_$shp" <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "f16x2" in r.get("Kernel_Name", ""):
            d[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[1].split("/")[-1], {k: [round(x / 1e6, 3) for x in v] for k, v in d.items()})
PY
  done
done
cd "$R"
for lib in libgnnea_eg1.so libgnnea.so libgnnea_eg8.so libgnnea.so; do
  GNNEA_LIB_FILE=$lib step "sk_${lib%.so}" 200 python -c "
import json, torch, bench
r = bench.sinkhorn_large(torch.device('cuda', 0))
print(json.dumps({'lib': '$lib', 'rate': r['iters_per_s']}))"
done
step casts5 600 python -u tools/dbg/cast_trace.py 2000000
echo done
