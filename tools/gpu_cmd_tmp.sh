set -o pipefail
mkdir -p gpurun_out
for m in 0 9 4 8 9; do GNNEA_X3P_MODE=$m timeout -k 10 100 python tools/dbg/x3_modes.py || exit 1; done
