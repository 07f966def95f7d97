timeout -k 10 200 python tools/dbg/x3p_check.py > gpurun_out/x3p_check.log 2>&1 || exit 1
GNNEA_X3P_NW=8 timeout -k 10 200 python tools/dbg/x3p_check.py > gpurun_out/x3p_check8.log 2>&1 || exit 1
for nw in 4 8; do for m in 0 2; do GNNEA_X3P_NW=$nw GNNEA_X3P_MODE=$m timeout -k 10 100 python tools/dbg/x3_modes.py | sed "s/^/nw $nw /" || exit 1; done; done
bash tools/gpu_cmd_tmp.sh
