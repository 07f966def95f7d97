#!/bin/bash
# PMC passes over tools/dbg/x3_only.py (x3 projection GEMM at cfg-4 shape): MFMA busy, waits, LDS.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/x3pmc
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
i=0
for pmc in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA" \
           "SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_LEVEL_WAVES SQ_WAVES SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VALU SQ_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_LDS SQ_THREAD_CYCLES_VALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $pmc -d "$O/p$i" -o run --output-format csv \
    -- python "$R/tools/dbg/x3_only.py" > "$O/p$i.log" 2>&1 || exit $?
done
python - "$O" <<'PY'
import csv, glob, sys, statistics
out = {}
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "gemm_x3" not in k:
            continue
        key = ("x3p" if "x3p" in k else "x3") + ":" + r["Counter_Name"]
        out.setdefault(key, []).append(float(r["Counter_Value"]))
for k in sorted(out):
    print(k, statistics.median(out[k]))
PY
