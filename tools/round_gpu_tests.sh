# Round-end GPU check, part 1: the whole -m gpu suite and smoke() (logs under gpurun_out/).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/gpu_all.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
tail -2 gpurun_out/smoke.log
