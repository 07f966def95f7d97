cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES -d $R/gpurun_out/pmc_sk1 -o run --output-format csv -- python3 $R/tools/microbench.py --n 1000 --only sinkhorn --reps 1 --out $R/gpurun_out/mb_pmc.json > $R/gpurun_out/pmc_sk1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_sk2 -o run --output-format csv -- python3 $R/tools/microbench.py --n 1000 --only sinkhorn --reps 1 --out $R/gpurun_out/mb_pmc.json > $R/gpurun_out/pmc_sk2.log 2>&1 || exit $?
echo done
