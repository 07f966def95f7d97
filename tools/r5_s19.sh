#!/bin/bash
# f16x2 GEMM with balanced column tiles: range tests, A/B timings, FETCH_SIZE
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/s20
mkdir -p "$O"
cd "$R"
step() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
step range 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_gemm_range.py
step ab 500 python -u tools/dbg/gemm_ab.py libgnnea_nonts.so libgnnea.so libgnnea_nonts.so libgnnea.so
cd /tmp && export TMPDIR=/tmp
for lib in libgnnea_nonts.so libgnnea.so; do
  for shp in proj proj600 dx; do
    GNNEA_LIB_FILE=$lib timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_${lib%.so}_$shp" -o run --output-format csv \
      -- python3 "$R/tools/dbg/gemm_one.py" $shp 3 > "$O/pmc_${lib%.so}_$shp.log" 2>&1 || exit 1
    python3 - "$O/pmc_${lib%.so}_$shp" <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "f16x2_ring" in r.get("Kernel_Name", ""):
            d[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[1].split("/")[-1], {k: [round(x / 1e6, 3) for x in v] for k, v in d.items()})
PY
  done
done
echo done
