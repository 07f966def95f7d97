#!/bin/bash
# PMC passes of the fused log-domain Sinkhorn sweep at B = 15000 (k_lsk_sweep):
# one counter set per rocprofv3 run (separate passes), 100 KNOPP iterations on the default path.
#   bash tools/sk_pmc15k.sh [outdir]
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=${1:-$R/gpurun_out/skpmc}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$name" -o run \
    --output-format csv -- python3 "$R/tools/sk_one.py" 15000 3 100 > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
pass p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_INSTS_VALU SQ_ACTIVE_INST_VALU || exit $?
pass p2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD \
  SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC || exit $?
pass p3 FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
pass p4 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 \
  SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT || true
echo done
