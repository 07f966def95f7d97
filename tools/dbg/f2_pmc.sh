#!/bin/bash
# PMC passes over tools/dbg/gemm_one.py proj (2M x 300 x 300) for the f16x2 ring (GNNEA_X3W=4) and
# the x3 ring (GNNEA_X3W=2): issue / wait split, MFMA busy, HBM bytes, L2 hits, clock.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/f2pmc
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for mode in 4 2; do
  i=0
  for pmc in "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD" \
             "FETCH_SIZE GRBM_GUI_ACTIVE" \
             "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
             "SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_LEVEL_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES"; do
    i=$((i+1))
    GNNEA_X3W=$mode timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $pmc -d "$O/m${mode}_p$i" -o run --output-format csv \
      -- python "$R/tools/dbg/gemm_one.py" proj 3 > "$O/m${mode}_p$i.log" 2>&1 || exit $?
  done
done
python - "$O" <<'PY'
import csv, glob, sys, statistics, json, os
out = {}
for f in glob.glob(sys.argv[1] + "/m*_p*/**/*counter_collection.csv", recursive=True):
    mode = os.path.relpath(f, sys.argv[1]).split("_")[0]
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "gemm" not in k or "pack" in k or "colscale" in k:
            continue
        out.setdefault(mode, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
res = {m: {c: statistics.median(v) for c, v in d.items()} for m, d in out.items()}
print(json.dumps(res, indent=1))
json.dump(res, open(sys.argv[1] + "/summary.json", "w"), indent=1)
PY
