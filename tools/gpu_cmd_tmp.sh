set -o pipefail
for m in 0 11 0 11; do GNNEA_X3P_MODE=$m timeout -k 10 100 python tools/dbg/x3_modes.py 2>&1 | grep -v amdgpu.ids || exit 1; done
GNNEA_X3P_MODE=11 timeout -k 10 200 python tools/dbg/x3p_big.py 2>&1 | grep -v amdgpu.ids || exit 1
