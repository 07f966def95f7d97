set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_sliced.py tests/test_gpu_parity.py -x -q -k "gat" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gat_t.log 2>&1 || { tail -5 gpurun_out/gat_t.log; exit 1; }
tail -1 gpurun_out/gat_t.log
rm -rf gpurun_out/prof_dl
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dl -o run --output-format csv -- python -u tools/dist_step.py --model GAT --steps 3 --warmup 1 > gpurun_out/prof_dl.log 2>&1 || exit 1
f=$(find gpurun_out/prof_dl -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/gat_kstats.csv
python - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/gat_kstats.csv")):
    if "k_gat_bwd" in r["Name"]:
        print(r["Name"][:44], "%.3f ms" % (float(r["AverageNs"])/1e6))
PY
timeout -k 10 300 python -u tools/dist_step.py --model GAT --steps 5 --warmup 2 2>/dev/null | tail -1 > gpurun_out/gat_step.json
cut -c1-330 gpurun_out/gat_step.json
