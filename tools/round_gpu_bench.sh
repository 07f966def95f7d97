# Round-end GPU check, part 2: the default bench line and the rocprofv3 evidence
# (kernel-trace stats + PMC passes of the headline SpMM, tools/prof_sliced.sh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python bench.py > gpurun_out/bench.log 2>&1 || exit 1
tail -1 gpurun_out/bench.log > gpurun_out/bench_line.json
rm -rf gpurun_out/prof_b gpurun_out/pmc_1 gpurun_out/pmc_2 gpurun_out/pmc_3
bash tools/prof_sliced.sh > gpurun_out/prof_sliced.log 2>&1 || exit 1
cat gpurun_out/spmm_pmc.json
