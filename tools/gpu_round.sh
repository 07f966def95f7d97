#!/bin/bash
# One GPU session on the MI355X box: parity tests, bench, rocprof kernel trace.
#   bash tools/gpu_round.sh [steps...]     steps: tests bench prof pmc smoke (default: tests bench prof)
# Every GPU step runs under its own time limit; a timeout / abort / segfault ends the session.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
steps=${*:-tests bench prof}

run() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/session.log"
  ( cd "$ROOT" && timeout -k 10 "$t" "$@" ) > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/session.log"
  tail -n 5 "$OUT/$name.log"
  case $rc in 124|137|134|139) echo "fatal rc=$rc in $name: stopping"; exit $rc ;; esac
  return 0
}

for s in $steps; do
  case $s in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider ;;
    bench) run bench 600 python bench.py ;;
    micro) run microbench 600 python tools/microbench.py ;;
    prof)
      ( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run \
          --output-format csv -- python "$ROOT/bench.py" --steps 10 --warmup 2 \
          --no-cpu-baseline ) > "$OUT/prof.log" 2>&1
      rc=$?; echo "== prof rc=$rc"; tail -n 3 "$OUT/prof.log"
      case $rc in 124|137|134|139) exit $rc ;; esac ;;
    gat5|gat4|hgcn)  # kernel trace of one EA training-step run (tools/dist_step.py)
      case $s in
        gat5) a="--model GAT --dtype bf16 --entities 2000000" ;;
        gat4) a="--model GAT" ;;
        hgcn) a="--model HGCN" ;;
      esac
      ( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$s" -o run \
          --output-format csv -- python "$ROOT/tools/dist_step.py" $a --steps 21 --warmup 3 ) \
          > "$OUT/prof_$s.log" 2>&1
      rc=$?; echo "== prof_$s rc=$rc"; tail -n 2 "$OUT/prof_$s.log"
      case $rc in 124|137|134|139) exit $rc ;; esac ;;
    pmc)
      ( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch" \
          -o run --output-format csv -- python "$ROOT/bench.py" --steps 3 --warmup 1 \
          --no-cpu-baseline --no-sinkhorn ) > "$OUT/pmc_fetch.log" 2>&1
      rc=$?; echo "== pmc fetch rc=$rc"; case $rc in 124|137|134|139) exit $rc ;; esac
      ( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_write" \
          -o run --output-format csv -- python "$ROOT/bench.py" --steps 3 --warmup 1 \
          --no-cpu-baseline --no-sinkhorn ) > "$OUT/pmc_write.log" 2>&1
      rc=$?; echo "== pmc write rc=$rc"; case $rc in 124|137|134|139) exit $rc ;; esac ;;
  esac
done
echo "session done"
