set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sliced.py -x -q -k "gat" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gatbwd.log 2>&1; rc=$?; tail -15 gpurun_out/gatbwd.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/dist_step.py --model GAT --steps 5 --warmup 2 > gpurun_out/gat_step.json 2> gpurun_out/gat_step.err || exit 1
tail -1 gpurun_out/gat_step.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gat -o run --output-format csv -- python -u tools/dist_step.py --model GAT --steps 3 --warmup 1 > gpurun_out/prof_gat.log 2>&1 || exit 1
f=$(find gpurun_out/prof_gat -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/gat_kstats.csv; head -25 $f | cut -c1-220
