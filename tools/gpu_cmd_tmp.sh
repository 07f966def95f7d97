set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof_dl
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dl -o run --output-format csv -- python -u tools/dist_step.py --model GAT --steps 3 --warmup 1 > gpurun_out/prof_dl.log 2>&1 || exit 1
f=$(find gpurun_out/prof_dl -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/gat_kstats.csv
python - <<'PY'
import csv
tot=0
for r in csv.DictReader(open("gpurun_out/gat_kstats.csv")):
    tot+=float(r["TotalDurationNs"])
    if "gnnea" in r["Name"]:
        print(r["Name"][:46], r["Calls"], "%.3f ms" % (float(r["AverageNs"])/1e6))
print("total kernel ms per step", tot/1e6/4)
PY
for i in 1 2; do timeout -k 10 300 python -u tools/dist_step.py --model GAT --steps 5 --warmup 2 2>/dev/null | tail -1 | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])"; done
